# Round 6 (session 2): ResNet-20 B=256 kernel table + step timeline of the final tree
set -o pipefail
O=gpurun_out/${1:-r6s2p}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --model resnet20 --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
cd $GRAFT_REPO_ROOT
python3 scripts/kstats.py $O/prof/run_kernel_stats.csv > $O/kstats.txt && cat $O/kstats.txt
python3 scripts/timeline.py $O/prof/run_kernel_trace.csv imgconv1_kernel 60 > $O/timeline.txt && tail -3 $O/timeline.txt
