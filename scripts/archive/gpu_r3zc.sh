# 128-deep k-tile glds GEMM tiles (19 / 20 / 21): layout + epilogue tests, fc1 GEMM sweep, CNN step A/B
# of the fc1 forward tile (DTFE_CNN_TILES).
set -o pipefail
O=gpurun_out/r3zc
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gemm_glds_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -1 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit $rc; }
timeout -k 10 300 python3 bench/gemm_sweep.py --iters 20 --tiles 8,12,14,19,20,21 > $O/sweep.txt 2>&1 || { tail -5 $O/sweep.txt; exit 1; }
cat $O/sweep.txt
for r in 1 2 3; do
  for v in 8,12,12 19,12,12 21,12,12 20,12,12; do
    DTFE_CNN_TILES=$v timeout -k 10 120 python3 bench.py > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
    echo "$v $(grep -o '"ms_per_step": [0-9.]*' $O/b.log)"
  done
done
exit 0
