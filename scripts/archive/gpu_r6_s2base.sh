# Round 6 (session 2) baseline on a fresh box: full GPU suite, every bench row, CNN in-graph timeline,
# ResNet-20 kernel table.  Usage: gpurun -- bash scripts/gpu_r6_s2base.sh <tag>
set -o pipefail
O=gpurun_out/${1:-r6s2base}
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -30; exit $rc; }
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for pw in 150 0; do
  timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --prewarm_ms $pw > $O/cnn_pw$pw.log 2>&1 || { tail -5 $O/cnn_pw$pw.log; exit 1; }
  echo "cnn prewarm=$pw $(grep -o '"ms_per_step": [0-9.]*' $O/cnn_pw$pw.log)"
done
timeout -k 10 200 python3 bench.py --model resnet20 --steps 20 --warmup 5 > $O/r20.log 2>&1 || { tail -5 $O/r20.log; exit 1; }
echo "r20 $(grep -o '"ms_per_step": [0-9.]*' $O/r20.log)"
timeout -k 10 300 python3 bench.py --model resnet50 --steps 20 --warmup 5 > $O/r50.log 2>&1 || { tail -5 $O/r50.log; exit 1; }
echo "r50 $(grep -o '"ms_per_step": [0-9.]*' $O/r50.log)"
timeout -k 10 200 python3 bench.py --dtype fp32 --steps 20 --warmup 5 > $O/cnn32.log 2>&1 || { tail -5 $O/cnn32.log; exit 1; }
echo "cnn fp32 $(grep -o '"ms_per_step": [0-9.]*' $O/cnn32.log)"
timeout -k 10 200 python3 bench/ref_models.py > $O/ref.log 2>&1 || { tail -5 $O/ref.log; exit 1; }
cat $O/ref.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof20 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --model resnet20 --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/$O/prof20.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$O/prof20.log; exit 1; }
cd $GRAFT_REPO_ROOT
python3 scripts/timeline.py $(ls $O/prof/*/run_kernel_trace.csv $O/prof/run_kernel_trace.csv 2>/dev/null | head -1) conv1c_fwd 15 > $O/timeline.txt && cat $O/timeline.txt
python3 scripts/kstats.py $(ls $O/prof20/*/run_kernel_stats.csv $O/prof20/run_kernel_stats.csv 2>/dev/null | head -1) > $O/kstats20.txt && head -40 $O/kstats20.txt
echo done
