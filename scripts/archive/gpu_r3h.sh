# fc1 GEMM pipeline-depth sweep (glds tiles 14..18) + CNN step A/B over the fc1 tile choice + step timeline.
set -o pipefail
O=gpurun_out/r3h
mkdir -p $O
timeout -k 10 120 python3 -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "gemm" --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench/gemm_sweep.py --iters 20 --tiles 8,12,14,15,16,17,18 > $O/sweep.log 2>&1; cat $O/sweep.log
for r in 1 2; do
  for t in 8,12,12 16,12,12 15,12,12 16,14,14 16,17,17 15,14,12; do
    DTFE_CNN_TILES=$t timeout -k 10 120 python3 bench.py --steps 200 --warmup 20 > $O/b_$t.log 2>&1 || { echo "bench $t failed"; tail -5 $O/b_$t.log; exit 1; }
    echo "tiles=$t $(grep -o '"ms_per_step": [0-9.]*' $O/b_$t.log)"
  done
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 30 --warmup 5 > $O/prof.log 2>&1 || exit 1
f=$(find $O/prof -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && python3 scripts/kstats.py "$f" > $O/kernels.txt && cat $O/kernels.txt
f=$(find $O/prof -name "*kernel_trace.csv" | head -1)
[ -n "$f" ] && python3 scripts/timeline.py "$f" conv1c_fwd > $O/timeline.txt && cat $O/timeline.txt
exit 0
