# Round 5: ps data-plane checks (bitwise reply test, bucket refresh, crash test without
# --heartbeat_secs) and the ps apply stream variants on the shared GPU (1 ps + 1 / 2 workers).
set -o pipefail
O=gpurun_out/${1:-r5ps}
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_cluster_gpu.py > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -30; exit $rc; }
for r in 1 2; do
  for st in normal high cu32 cu64; do
    timeout -k 10 240 python3 bench.py --mode ps --gpus 1 --steps 200 --warmup 20 --ps_stream $st > $O/ps11_${st}_$r.log 2>&1 || { tail -5 $O/ps11_${st}_$r.log; exit 1; }
    echo "ps11 $st $r $(grep -o '"value": [0-9.]*' $O/ps11_${st}_$r.log) $(grep -o '"ms_per_step": [0-9.]*' $O/ps11_${st}_$r.log)"
  done
done
for st in normal high; do
  timeout -k 10 240 python3 bench.py --mode ps --gpus 2 --steps 200 --warmup 20 --ps_stream $st > $O/ps12_$st.log 2>&1 || { tail -5 $O/ps12_$st.log; exit 1; }
  echo "ps12 $st $(grep -o '"value": [0-9.]*' $O/ps12_$st.log) $(grep -o '"ms_per_step": [0-9.]*' $O/ps12_$st.log) $(grep -o '"ps_refreshed_ranges": [0-9]*' $O/ps12_$st.log)"
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for st in normal high; do
  DTFE_PROFILE_EXIT=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_ps_$st -o run_%pid% -- python3 bench.py --mode ps --gpus 1 --steps 40 --warmup 10 --ps_stream $st > $O/prof_ps_$st.log 2>&1 || { tail -5 $O/prof_ps_$st.log; exit 1; }
  python3 scripts/ps_timeline.py $O/prof_ps_$st > $O/ps_timeline_$st.txt 2>&1; grep -i "median\|apply" $O/ps_timeline_$st.txt | head -8
done
