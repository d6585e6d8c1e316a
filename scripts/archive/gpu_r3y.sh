# conv2 data gradient captured before the weight gradient (same fork point) vs the default order.
set -o pipefail
O=gpurun_out/r3y
mkdir -p $O
DTFE_CNN_DGRAD_FIRST=1 timeout -k 10 300 python3 -u -m pytest tests/test_mnist_cnn_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -1 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit $rc; }
for r in 1 2 3; do
  for v in 0 1; do
    DTFE_CNN_DGRAD_FIRST=$v timeout -k 10 120 python3 bench.py > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
    echo "dgrad_first=$v $(grep -o '"ms_per_step": [0-9.]*' $O/b.log)"
  done
done
export DTFE_CNN_DGRAD_FIRST=1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 30 --warmup 5 > $O/prof.log 2>&1 || exit 1
f=$(find $O/prof -name "*kernel_trace.csv" | head -1)
[ -n "$f" ] && python3 scripts/timeline.py "$f" conv1c_fwd > $O/timeline.txt && cat $O/timeline.txt
exit 0
