# BN-backward statistics from the data-gradient epilogue: kernel tests, ResNet tests, A/B bench, fp32 trajectory.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_resnet.py -m gpu -x -v --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/bb_tests.log 2>&1 &&
DTFE_BN_BWD_FUSE=0 timeout -k 10 200 python3 bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/bb_off.log 2>&1 &&
DTFE_BN_BWD_FUSE=1 timeout -k 10 200 python3 bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/bb_on.log 2>&1 &&
DTFE_BN_BWD_FUSE=0 timeout -k 10 200 python3 bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/bb_off2.log 2>&1 &&
DTFE_BN_BWD_FUSE=1 timeout -k 10 200 python3 bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/bb_on2.log 2>&1 &&
timeout -k 10 300 python3 scripts/r50_train_compare.py --batch 256 --steps 12 > gpurun_out/bb_train_cmp.log 2>&1
rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/bb_tests.log | tail -20
for f in bb_off bb_on bb_off2 bb_on2; do python3 -c "import json; r=json.loads(open('gpurun_out/$f.log').read().strip().splitlines()[-1]); print('$f', r['ms_per_step'], r['median_window_ms_per_step'], r['config']['last_loss'])" || tail -5 gpurun_out/$f.log; done
tail -13 gpurun_out/bb_train_cmp.log
exit $rc
