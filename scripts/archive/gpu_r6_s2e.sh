# Round 6 (session 2): fp32 conv1 kernels (1-channel forward, pooled weight gradient) - tests, fp32 bench, profile
set -o pipefail
O=gpurun_out/${1:-r6s2e}
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_kernels_gpu.py tests/test_mnist_cnn_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu -k "conv or fp32 or cnn or head" > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -30; exit $rc; }
for i in 1 2; do
timeout -k 10 200 python3 bench.py --dtype fp32 --steps 20 --warmup 5 > $O/cnn32_$i.log 2>&1 || { tail -5 $O/cnn32_$i.log; exit 1; }
echo "cnn fp32 $(grep -o '"ms_per_step": [0-9.]*' $O/cnn32_$i.log) $(grep -o '"value": [0-9.]*' $O/cnn32_$i.log)"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof32 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --dtype fp32 --steps 10 --warmup 3 > $GRAFT_REPO_ROOT/$O/prof32.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$O/prof32.log; exit 1; }
cd $GRAFT_REPO_ROOT
python3 scripts/timeline.py $O/prof32/run_kernel_trace.csv gather_rows 8 > $O/timeline32.txt && cat $O/timeline32.txt
