# Round 6 (session 2): MNIST-CNN Adam work order (tiles first) and conv2 wgrad grid A/B; timeline
set -o pipefail
O=gpurun_out/${1:-r6s2d}
mkdir -p $O
timeout -k 10 500 python3 bench/cnn_ab.py --arms "optim.TILES_FIRST=1" "optim.TILES_FIRST=0" "c2_blocks=160" "c2_blocks=224" "c2_blocks=256" --rounds 2 > $O/ab.log 2>&1 || { tail -5 $O/ab.log; exit 1; }
grep ms/step $O/ab.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof32 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --dtype fp32 --steps 10 --warmup 3 > $GRAFT_REPO_ROOT/$O/prof32.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$O/prof32.log; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/profref -o run -- python3 $GRAFT_REPO_ROOT/bench/ref_models.py > $GRAFT_REPO_ROOT/$O/profref.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$O/profref.log; exit 1; }
cd $GRAFT_REPO_ROOT
python3 scripts/timeline.py $(ls $O/prof/*/run_kernel_trace.csv $O/prof/run_kernel_trace.csv 2>/dev/null | head -1) conv1c_fwd 15 > $O/timeline.txt && cat $O/timeline.txt
python3 scripts/kstats.py $(ls $O/prof32/run_kernel_stats.csv) > $O/kstats32.txt && cat $O/kstats32.txt
python3 scripts/kstats.py $(ls $O/profref/run_kernel_stats.csv) > $O/kstatsref.txt && cat $O/kstatsref.txt
