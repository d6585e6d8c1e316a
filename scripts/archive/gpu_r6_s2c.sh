# Round 6 (session 2): MNIST-CNN fc/head Adam on a side branch (LDS-free apply) - tests, A/B, timeline
set -o pipefail
O=gpurun_out/${1:-r6s2c}
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_mnist_cnn_gpu.py tests/test_models_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -30; exit $rc; }
timeout -k 10 400 python3 bench/cnn_ab.py --arms "side_adam=1" "side_adam=0" "side_adam=1,side_blocks=128" "side_adam=1,side_blocks=512" --rounds 2 > $O/ab.log 2>&1 || { tail -5 $O/ab.log; exit 1; }
grep ms/step $O/ab.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
cd $GRAFT_REPO_ROOT
python3 scripts/timeline.py $(ls $O/prof/*/run_kernel_trace.csv $O/prof/run_kernel_trace.csv 2>/dev/null | head -1) conv1c_fwd 15 > $O/timeline.txt && cat $O/timeline.txt
