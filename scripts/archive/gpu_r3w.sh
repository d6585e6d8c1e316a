# ResNet-50 weight-gradient implicit GEMM with three LDS stages (DTFE_IGW_NST=3) vs two: numerics
# (GPU conv tests under NST=3), per-layer conv times, and the B=256 training step, alternating.
set -o pipefail
O=gpurun_out/r3w
mkdir -p $O
DTFE_IGW_NST=3 timeout -k 10 400 python3 -u -m pytest tests/test_resnet.py tests/test_igemm_gpu.py tests/test_igemm_tiles_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit $rc; }
for n in 2 3; do
  DTFE_IGW_NST=$n timeout -k 10 300 python3 bench/resnet50_convs.py --batch 256 --reps 10 --no-torch > $O/convs_$n.txt 2>&1 || { tail -5 $O/convs_$n.txt; exit 1; }
  echo "NST=$n"; grep -E "totals" $O/convs_$n.txt
done
for r in 1 2; do
  for n in 2 3; do
    DTFE_IGW_NST=$n timeout -k 10 300 python3 bench.py --model resnet50 --steps 20 --warmup 5 > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
    echo "NST=$n $(grep -o '"value": [0-9.]*' $O/b.log) $(grep -o '"ms_per_step": [0-9.]*' $O/b.log)"
  done
done
exit 0
