# Round 5: ResNet-20 (B=256) step time and kernel trace (kernel table + launch count)
set -o pipefail
O=gpurun_out/${1:-r5r20}
mkdir -p $O
timeout -k 10 200 python3 bench.py --model resnet20 --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' $O/bench.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --model resnet20 --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
echo done
