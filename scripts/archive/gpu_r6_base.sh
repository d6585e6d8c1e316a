# Round 6 baseline on a fresh box: CNN bench (pre-warmed / cold), in-graph CNN kernel trace,
# fc1 GEMM sweep.  Usage: gpurun -- bash scripts/gpu_r6_base.sh <tag>
set -o pipefail
O=gpurun_out/${1:-r6base}
mkdir -p $O
for pw in 150 0; do
  timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --prewarm_ms $pw > $O/cnn_pw$pw.log 2>&1 || { tail -5 $O/cnn_pw$pw.log; exit 1; }
  echo "cnn prewarm=$pw $(grep -o '"ms_per_step": [0-9.]*' $O/cnn_pw$pw.log)"
done
timeout -k 10 200 python3 bench/gemm_sweep.py --iters 20 --tiles 12,19 --splits 1 > $O/gemm.log 2>&1 || { tail -5 $O/gemm.log; exit 1; }
cat $O/gemm.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
cd $GRAFT_REPO_ROOT
python3 scripts/timeline.py $(ls $O/prof/*/run_kernel_trace.csv | head -1) conv1c_fwd 15 > $O/timeline.txt && cat $O/timeline.txt
echo done
