# head wgrad butterfly kernel + conv1 fwd compile-time act; conv1 wgrad grid sweep; step timeline.
set -o pipefail
O=gpurun_out/r3j
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_kernels_gpu.py tests/test_imgconv.py tests/test_mnist_cnn_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit $rc; }
timeout -k 10 120 python3 bench/cnn_kernels.py --iters 30 --only conv1_fwd,head,head_wgrad,head_wgrad_k,conv1_wgrad > $O/k.log 2>&1; cat $O/k.log
for r in 1 2; do
  for g in 256 512 1024; do
    DTFE_C1W_GRID=$g timeout -k 10 120 python3 bench.py > $O/b_$g.log 2>&1 || exit 1; echo "c1w_grid=$g $(grep -o '"ms_per_step": [0-9.]*' $O/b_$g.log)"
  done
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 30 --warmup 5 > $O/prof.log 2>&1 || exit 1
f=$(find $O/prof -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && python3 scripts/kstats.py "$f" > $O/kernels.txt && cat $O/kernels.txt
f=$(find $O/prof -name "*kernel_trace.csv" | head -1)
[ -n "$f" ] && python3 scripts/timeline.py "$f" conv1c_fwd > $O/timeline.txt && cat $O/timeline.txt
exit 0
