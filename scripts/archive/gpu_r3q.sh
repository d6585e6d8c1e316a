# conv2 weight gradient software pipeline: kernel tests, rocprof kernel time and step A/B vs the previous
# imgwgrad_persist.hip (A/B library _C/ab via DTFE_KERNEL_LIB).
set -o pipefail
O=gpurun_out/r3q
mkdir -p $O
OLD=distributed-tensorflow-examples_amd/_C/ab/libdtfe_kernels.so
timeout -k 10 300 python3 -u -m pytest tests/test_imgconv.py tests/test_mnist_cnn_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit $rc; }
bash scripts/abl.sh $O DTFE_IW_DIAG "0 4" conv2_wgrad_ws imgwgrad_persist || exit 1
( export DTFE_KERNEL_LIB=$OLD; bash scripts/abl.sh $O/old DTFE_IW_DIAG "0" conv2_wgrad_ws imgwgrad_persist ) || exit 1
for r in 1 2 3; do
  for lib in new old; do
    if [ $lib = old ]; then export DTFE_KERNEL_LIB=$OLD; else unset DTFE_KERNEL_LIB; fi
    timeout -k 10 120 python3 bench.py > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
    echo "wgrad=$lib $(grep -o '"ms_per_step": [0-9.]*' $O/b.log)"
  done
done
unset DTFE_KERNEL_LIB
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 30 --warmup 5 > $O/prof.log 2>&1 || exit 1
f=$(find $O/prof -name "*kernel_trace.csv" | head -1)
[ -n "$f" ] && python3 scripts/timeline.py "$f" conv1c_fwd > $O/timeline.txt && cat $O/timeline.txt
exit 0
