# Round 6: ResNet-20 two ranks on one GPU (gloo + IPC all-reduce): bench line + per-rank kernel table
set -o pipefail
O=gpurun_out/${1:-r6r20x2}
mkdir -p $O
timeout -k 10 300 python3 bench.py --model resnet20 --gpus 2 --backend gloo --comm ipc --steps 20 --warmup 5 > $O/r20x2.log 2>&1 || { tail -5 $O/r20x2.log; exit 1; }
tail -1 $O/r20x2.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --model resnet20 --gpus 2 --backend gloo --comm ipc --steps 10 --warmup 3 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
cd $GRAFT_REPO_ROOT
ls -R $O/prof | head -20
