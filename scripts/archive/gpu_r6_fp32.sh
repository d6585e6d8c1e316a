# Round 6: reference-precision rows - fp32 CNN kernel table, LSTM / GAN / encoder steps
set -o pipefail
O=gpurun_out/${1:-r6fp32}
mkdir -p $O
timeout -k 10 200 python3 bench.py --dtype fp32 --steps 30 --warmup 5 > $O/cnn32.log 2>&1 || { tail -5 $O/cnn32.log; exit 1; }
tail -1 $O/cnn32.log
timeout -k 10 300 python3 bench/ref_models.py > $O/ref.log 2>&1 || { tail -5 $O/ref.log; exit 1; }
cat $O/ref.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --dtype fp32 --steps 10 --warmup 3 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_lstm -o run -- python3 $GRAFT_REPO_ROOT/bench/ref_models.py --models lstm > $GRAFT_REPO_ROOT/$O/prof_lstm.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$O/prof_lstm.log; exit 1; }
cd $GRAFT_REPO_ROOT
python3 -c "
import csv,sys
for f in sys.argv[1:]:
    rows=list(csv.DictReader(open(f)))
    rows.sort(key=lambda r:-float(r['TotalDurationNs']))
    print('==',f)
    for r in rows[:25]: print('%10.1f us x %5s  %8.2f avg  %s'%(float(r['TotalDurationNs'])/1e3, r['Calls'], float(r['AverageNs'])/1e3, r['Name'][:90]))
" $O/prof/run_kernel_stats.csv $O/prof_lstm/run_kernel_stats.csv
