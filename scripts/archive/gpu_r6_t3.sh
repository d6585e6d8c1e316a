# Round 6: glds DMA from inline asm (no compiler vmcnt(0) before the tr reads): GEMM tests, CNN tests,
# fc1 sweep, CNN bench + in-graph trace
set -o pipefail
O=gpurun_out/${1:-r6t3}
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gemm_glds_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gemm.log 2>&1
rc=$?; tail -3 $O/pytest_gemm.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest_gemm.log | head -30; exit $rc; }
timeout -k 10 300 python3 -u -m pytest tests/test_mnist_cnn_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_cnn.log 2>&1
rc=$?; tail -3 $O/pytest_cnn.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest_cnn.log | head -30; exit $rc; }
timeout -k 10 200 python3 bench/gemm_sweep.py --iters 20 --tiles 12,19,22 --splits 1 > $O/gemm.log 2>&1 || { tail -5 $O/gemm.log; exit 1; }
cat $O/gemm.log
for pw in 150 0; do
  timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --prewarm_ms $pw > $O/cnn_pw$pw.log 2>&1 || { tail -5 $O/cnn_pw$pw.log; exit 1; }
  echo "cnn prewarm=$pw $(grep -o '"ms_per_step": [0-9.]*' $O/cnn_pw$pw.log)"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
cd $GRAFT_REPO_ROOT
python3 scripts/timeline.py $(ls $O/prof/*kernel_trace.csv | head -1) conv1c_fwd 15 > $O/timeline.txt && cat $O/timeline.txt
