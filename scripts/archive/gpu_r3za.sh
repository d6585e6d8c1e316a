# New default order (conv2 dgrad captured first, wgrad 192 WGs): fc/head Adam placement A/B
# (DTFE_CNN_FC_APPLY join | main | c2) + GPU tests of the CNN.
set -o pipefail
O=gpurun_out/r3za
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_mnist_cnn_gpu.py tests/test_imgconv.py -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -1 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit $rc; }
for r in 1 2 3; do
  for v in join main c2; do
    DTFE_CNN_FC_APPLY=$v timeout -k 10 120 python3 bench.py > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
    echo "$v $(grep -o '"ms_per_step": [0-9.]*' $O/b.log)"
  done
done
export DTFE_CNN_FC_APPLY=main
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 30 --warmup 5 > $O/prof.log 2>&1 || exit 1
f=$(find $O/prof -name "*kernel_trace.csv" | head -1)
[ -n "$f" ] && python3 scripts/timeline.py "$f" conv1c_fwd > $O/timeline.txt && cat $O/timeline.txt
exit 0
