# Round 6 (session 2): LSTM split recurrence over 8 CUs per row group (NS = 8) - tests, A/B vs NS = 4, profile
set -o pipefail
O=gpurun_out/${1:-r6s2l}
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_models_gpu.py tests/test_dense_head.py tests/test_resnet.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu -k "lstm or dense" > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -30; exit $rc; }
for ns in 8 8; do
  DTFE_LSTM_SPLIT=$ns timeout -k 10 200 python3 bench/ref_models.py --models lstm > $O/lstm_$ns.log 2>&1 || { tail -5 $O/lstm_$ns.log; exit 1; }
  echo "NS=$ns $(grep ms_per_step $O/lstm_$ns.log)"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench/ref_models.py --models lstm > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
cd $GRAFT_REPO_ROOT
python3 scripts/timeline.py $O/prof/run_kernel_trace.csv seq_stage 100 > $O/timeline.txt && cat $O/timeline.txt
