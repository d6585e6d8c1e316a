# BN partial reduce in one launch (last-arriver hand-off) vs two launches: tests, ResNet-50 A/B.
set -o pipefail
O=gpurun_out/bnpart
mkdir -p $O
DTFE_BN_PART_1L=1 timeout -k 10 400 python3 -u -m pytest tests/test_norm_gpu.py tests/test_resnet.py -m gpu -x -q --timeout 120 \
  --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 &&
DTFE_BN_PART_1L=0 timeout -k 10 200 python3 bench.py --model resnet50 --steps 20 --warmup 5 > $O/b_2l.log 2>&1 &&
DTFE_BN_PART_1L=1 timeout -k 10 200 python3 bench.py --model resnet50 --steps 20 --warmup 5 > $O/b_1l.log 2>&1 &&
DTFE_BN_PART_1L=0 timeout -k 10 200 python3 bench.py --model resnet50 --steps 20 --warmup 5 > $O/b_2l2.log 2>&1 &&
DTFE_BN_PART_1L=1 timeout -k 10 200 python3 bench.py --model resnet50 --steps 20 --warmup 5 > $O/b_1l2.log 2>&1 &&
timeout -k 10 200 python3 bench.py --model resnet20 > $O/b_r20.log 2>&1
rc=$?
tail -n 2 $O/tests.log
for f in b_2l b_1l b_2l2 b_1l2 b_r20; do python3 -c "import json; r=json.loads(open('$O/$f.log').read().strip().splitlines()[-1]); print('$f', r['ms_per_step'], r['median_window_ms_per_step'], r['config']['last_loss'])" || tail -3 $O/$f.log; done
exit $rc
