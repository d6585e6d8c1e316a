# Round 6: ResNet-20 fused statistics (butterfly fold) + fp32 conv weight-gradient loader: tests, benches, tables
set -o pipefail
O=gpurun_out/${1:-r6t10}
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_imgconv.py tests/test_resnet.py tests/test_kernels_gpu.py tests/test_mnist_cnn_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu -k "imgconv or resnet or wgrad or fp32" > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -30; exit $rc; }
timeout -k 10 200 python3 bench.py --model resnet20 --steps 30 --warmup 10 > $O/r20.log 2>&1 || { tail -5 $O/r20.log; exit 1; }
tail -1 $O/r20.log | cut -c1-300
timeout -k 10 200 python3 bench.py --dtype fp32 --steps 30 --warmup 5 > $O/cnn32.log 2>&1 || { tail -5 $O/cnn32.log; exit 1; }
tail -1 $O/cnn32.log | cut -c1-300
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --model resnet20 --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof32 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --dtype fp32 --steps 10 --warmup 3 > $GRAFT_REPO_ROOT/$O/prof32.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$O/prof32.log; exit 1; }
cd $GRAFT_REPO_ROOT
python3 scripts/kstats.py $O/prof/run_kernel_stats.csv > $O/kstats.txt && cat $O/kstats.txt
python3 scripts/kstats.py $O/prof32/run_kernel_stats.csv > $O/kstats32.txt && cat $O/kstats32.txt
