# Round 6: warp-specialized ring fc GEMM (tile 23) and the persistent conv's fused output BN statistics:
# tests, fc1 sweep vs tile 22, ResNet-20 bench + kernel table
set -o pipefail
O=gpurun_out/${1:-r6t7}
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_imgconv.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu > $O/pytest_imgconv.log 2>&1
rc=$?; tail -3 $O/pytest_imgconv.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest_imgconv.log | head -30; exit $rc; }
timeout -k 10 300 python3 -u -m pytest tests/test_gemm_glds_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "tile22_layouts and 23" > $O/pytest_ring.log 2>&1
rc=$?; tail -3 $O/pytest_ring.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest_ring.log | head -30; exit $rc; }
timeout -k 10 300 python3 -u -m pytest tests/test_gemm_glds_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gemm.log 2>&1
rc=$?; tail -3 $O/pytest_gemm.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest_gemm.log | head -30; exit $rc; }
timeout -k 10 200 python3 bench/gemm_sweep.py --iters 20 --tiles 12,22,23 --splits 1 > $O/gemm.log 2>&1 || { tail -5 $O/gemm.log; exit 1; }
cat $O/gemm.log
timeout -k 10 400 python3 -u -m pytest tests/test_resnet.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu > $O/pytest_resnet.log 2>&1
rc=$?; tail -3 $O/pytest_resnet.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest_resnet.log | head -30; exit $rc; }
timeout -k 10 200 python3 bench.py --model resnet20 --steps 30 --warmup 10 > $O/r20.log 2>&1 || { tail -5 $O/r20.log; exit 1; }
tail -1 $O/r20.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --model resnet20 --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
cd $GRAFT_REPO_ROOT
head -40 $O/prof/run_kernel_stats.csv
