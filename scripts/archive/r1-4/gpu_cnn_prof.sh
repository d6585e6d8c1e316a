# MNIST CNN: tests, headline bench, rocprofv3 kernel stats + one-step timeline
set -o pipefail
O=gpurun_out/${1:-r2i}
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_imgconv.py tests/test_mnist_cnn_gpu.py > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python3 bench.py --steps 200 --warmup 20 > $O/bench.log 2>&1 && grep '^{' $O/bench.log | cut -c1-260 || exit 1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_cnn -o run -- python3 bench.py --steps 30 --warmup 5 > $O/prof_cnn.log 2>&1 || exit 1
f=$(find $O/prof_cnn -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && python3 scripts/kstats.py "$f" > $O/cnn_kernels_prof.txt && cat $O/cnn_kernels_prof.txt
f=$(find $O/prof_cnn -name "*kernel_trace.csv" | head -1)
[ -n "$f" ] && python3 scripts/timeline.py "$f" conv1c_fwd > $O/cnn_timeline.txt && cat $O/cnn_timeline.txt
exit 0
