# Round 6: new ResNet-20 tests (evaluate at B=128, deferred-queue guard, bucket flush, bench-shaped
# step vs fp32) + the in-graph CNN kernel trace
set -o pipefail
O=gpurun_out/${1:-r6t1}
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_resnet.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider -k "fold_batch or queue_guard or grouped_flush or bucket_flush or bench_shaped or evaluate" > $O/pytest.log 2>&1
rc=$?; tail -15 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -30; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
cd $GRAFT_REPO_ROOT
python3 scripts/timeline.py $(ls $O/prof/*/run_kernel_trace.csv | head -1) conv1c_fwd 15 > $O/timeline.txt && cat $O/timeline.txt
exit $rc
