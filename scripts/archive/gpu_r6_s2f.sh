# Round 6 (session 2): LSTM head as one fused fp32 launch (generalised dense_head) - tests, ref-model times
set -o pipefail
O=gpurun_out/${1:-r6s2f}
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_dense_head.py tests/test_models_gpu.py tests/test_resnet.py -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -30; exit $rc; }
timeout -k 10 200 python3 bench.py --model resnet20 --steps 20 --warmup 5 > $O/r20.log 2>&1 || { tail -5 $O/r20.log; exit 1; }
echo "r20 $(grep -o "\"ms_per_step\": [0-9.]*" $O/r20.log)"
for i in 1 2; do
timeout -k 10 200 python3 bench/ref_models.py > $O/ref_$i.log 2>&1 || { tail -5 $O/ref_$i.log; exit 1; }
grep ms_per_step $O/ref_$i.log
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/profref -o run -- python3 $GRAFT_REPO_ROOT/bench/ref_models.py --models lstm > $GRAFT_REPO_ROOT/$O/profref.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$O/profref.log; exit 1; }
cd $GRAFT_REPO_ROOT
python3 scripts/kstats.py $O/profref/run_kernel_stats.csv > $O/kstatsref.txt && cat $O/kstatsref.txt
python3 scripts/timeline.py $O/profref/run_kernel_trace.csv seq_stage 100 > $O/timeline_lstm.txt && cat $O/timeline_lstm.txt
