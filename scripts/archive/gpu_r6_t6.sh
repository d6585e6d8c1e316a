# Round 6: conv1 kernels (aligned-read shifted copies, swizzled dY image, MFMA bias gradient): tests,
# isolated kernel times, CNN bench + in-graph trace
set -o pipefail
O=gpurun_out/${1:-r6t6}
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_mnist_cnn_gpu.py tests/test_imgconv.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -30; exit $rc; }
timeout -k 10 200 python3 bench/cnn_kernels.py --iters 30 > $O/kernels.log 2>&1 || { tail -5 $O/kernels.log; exit 1; }
cat $O/kernels.log
for pw in 150 0 150; do
  timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --prewarm_ms $pw > $O/cnn_pw$pw.log 2>&1 || { tail -5 $O/cnn_pw$pw.log; exit 1; }
  echo "cnn prewarm=$pw $(grep -o '"ms_per_step": [0-9.]*' $O/cnn_pw$pw.log)"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
cd $GRAFT_REPO_ROOT
python3 scripts/timeline.py $(ls $O/prof/*kernel_trace.csv | head -1) conv1c_fwd 15 > $O/timeline.txt && cat $O/timeline.txt
