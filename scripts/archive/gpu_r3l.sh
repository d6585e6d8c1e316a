# Grouped fc backward launch (head wgrad + fc1 dgrad + fc1 wgrad in one grid) A/B + timeline; fc1 PMC.
set -o pipefail
O=gpurun_out/r3l
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit $rc; }
for r in 1 2 3; do
  for g in 1 0; do
    DTFE_CNN_FC_GROUP=$g timeout -k 10 120 python3 bench.py > $O/b_$g.log 2>&1 || exit 1; echo "fc_group=$g $(grep -o '"ms_per_step": [0-9.]*' $O/b_$g.log)"
  done
done
timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 > $O/b_driver.log 2>&1 && grep -o '"ms_per_step": [0-9.]*' $O/b_driver.log
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 30 --warmup 5 > $O/prof.log 2>&1 || exit 1
f=$(find $O/prof -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && python3 scripts/kstats.py "$f" > $O/kernels.txt && cat $O/kernels.txt
f=$(find $O/prof -name "*kernel_trace.csv" | head -1)
[ -n "$f" ] && python3 scripts/timeline.py "$f" conv1c_fwd > $O/timeline.txt && cat $O/timeline.txt
bash scripts/gpu_r3k.sh
exit 0
