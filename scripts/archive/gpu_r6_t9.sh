# Round 6: ResNet-20 fused output statistics (inlined fold): tests, bench, kernel table
set -o pipefail
O=gpurun_out/${1:-r6t9}
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_imgconv.py tests/test_resnet.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -30; exit $rc; }
timeout -k 10 200 python3 bench.py --model resnet20 --steps 30 --warmup 10 > $O/r20.log 2>&1 || { tail -5 $O/r20.log; exit 1; }
tail -1 $O/r20.log | cut -c1-400
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --model resnet20 --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
cd $GRAFT_REPO_ROOT
python3 scripts/kstats.py $O/prof/run_kernel_stats.csv > $O/kstats.txt 2>&1 || python3 -c "
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r:-float(r['TotalDurationNs']))
for r in rows[:40]: print('%10.1f us x %5s  %8.2f avg  %s'%(float(r['TotalDurationNs'])/1e3, r['Calls'], float(r['AverageNs'])/1e3, r['Name'][:100]))
" $O/prof/run_kernel_stats.csv > $O/kstats.txt
cat $O/kstats.txt
