# One-replica branch apply with the conv Adam split in two (conv2 on its branch, conv1
# ending the main chain: no kernel after the join) vs the default whole apply.
set -o pipefail
O=gpurun_out/r3t
mkdir -p $O
OLD=distributed-tensorflow-examples_amd/_C/ab/libdtfe_kernels.so
timeout -k 10 400 python3 -u -m pytest tests/test_mnist_cnn_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit $rc; }
for r in 1 2 3; do
  for v in new branch; do
    unset DTFE_KERNEL_LIB DTFE_CNN_BRANCH_APPLY
    [ $v = old ] && export DTFE_KERNEL_LIB=$OLD
    [ $v = branch ] && export DTFE_CNN_BRANCH_APPLY=1
    timeout -k 10 120 python3 bench.py > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
    echo "$v $(grep -o '"ms_per_step": [0-9.]*' $O/b.log)"
  done
done
unset DTFE_KERNEL_LIB
export DTFE_CNN_BRANCH_APPLY=1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 30 --warmup 5 > $O/prof.log 2>&1 || exit 1
f=$(find $O/prof -name "*kernel_trace.csv" | head -1)
[ -n "$f" ] && python3 scripts/timeline.py "$f" conv1c_fwd > $O/timeline.txt && cat $O/timeline.txt
exit 0
