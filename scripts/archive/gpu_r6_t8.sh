# Round 6: ResNet-20 fused output statistics - gradient oracle per variable (fused vs bn_stats), bench,
# kernel table; then the fp32 rows (scripts/gpu_r6_fp32.sh)
set -o pipefail
O=gpurun_out/${1:-r6t8}
mkdir -p $O
timeout -k 10 200 python3 bench/r20_grad_cos.py > $O/r20cos.log 2>&1 || { tail -5 $O/r20cos.log; exit 1; }
cat $O/r20cos.log
timeout -k 10 200 python3 bench.py --model resnet20 --steps 30 --warmup 10 > $O/r20.log 2>&1 || { tail -5 $O/r20.log; exit 1; }
tail -1 $O/r20.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --model resnet20 --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
cd $GRAFT_REPO_ROOT
python3 -c "
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r:-float(r['TotalDurationNs']))
for r in rows[:40]: print('%10.1f us x %5s  %8.2f avg  %s'%(float(r['TotalDurationNs'])/1e3, r['Calls'], float(r['AverageNs'])/1e3, r['Name'][:90]))
" $O/prof/run_kernel_stats.csv
bash scripts/gpu_r6_fp32.sh ${1:-r6t8}_fp32
