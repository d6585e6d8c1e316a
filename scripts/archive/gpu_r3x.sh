# (1) MNIST conv1 weight gradient with the in-kernel two-level partial-sum reduce (default) vs the
#     separate reduce kernel (DTFE_C1W_FUSED_REDUCE=0): GPU tests + step A/B + timeline.
# (2) ResNet-50 weight-gradient implicit GEMM with three LDS stages (DTFE_IGW_NST=3) vs two.
set -o pipefail
O=gpurun_out/r3x
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_imgconv.py tests/test_mnist_cnn_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_cnn.log 2>&1
rc=$?; tail -1 $O/pytest_cnn.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest_cnn.log | head -20; exit $rc; }
for r in 1 2 3; do
  for v in 1 0; do
    DTFE_C1W_FUSED_REDUCE=$v timeout -k 10 120 python3 bench.py > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
    echo "c1w_fused=$v $(grep -o '"ms_per_step": [0-9.]*' $O/b.log)"
  done
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 30 --warmup 5 > $O/prof.log 2>&1 || exit 1
f=$(find $O/prof -name "*kernel_trace.csv" | head -1)
[ -n "$f" ] && python3 scripts/timeline.py "$f" conv1c_fwd > $O/timeline.txt && cat $O/timeline.txt
DTFE_IGW_NST=3 timeout -k 10 400 python3 -u -m pytest tests/test_resnet.py tests/test_igemm_gpu.py tests/test_igemm_tiles_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_r50.log 2>&1
rc=$?; tail -1 $O/pytest_r50.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest_r50.log | head -20; exit $rc; }
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
