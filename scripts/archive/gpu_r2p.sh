# BN statistics flush A/B on one box, interleaved: legacy (serial LDS sum + atomics) vs tree + atomics vs slots
set -o pipefail
O=gpurun_out/r2p
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_norm_gpu.py > $O/pytest.log 2>&1
rc=$?; tail -1 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do for m in "DTFE_BN_LEGACY=1" "DTFE_BN_LEGACY=0"; do
env $m timeout -k 10 240 python3 bench.py --model resnet20 --steps 100 --warmup 10 > $O/b.log 2>&1 && echo "$m $(grep '^{' $O/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["median_window_ms_per_step"])')" || exit 1
done; done
