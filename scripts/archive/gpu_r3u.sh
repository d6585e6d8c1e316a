# conv2 backward serial (DTFE_CNN_BRANCHES=fc: no fork / join in the step graph at all, both conv2
# backward kernels on the whole chip) vs the default concurrent branch.
set -o pipefail
O=gpurun_out/r3u
mkdir -p $O
for r in 1 2 3; do
  for v in fc,c2 fc; do
    export DTFE_CNN_BRANCHES=$v
    timeout -k 10 120 python3 bench.py > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
    echo "$v $(grep -o '"ms_per_step": [0-9.]*' $O/b.log)"
  done
done
export DTFE_CNN_BRANCHES=fc
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 30 --warmup 5 > $O/prof.log 2>&1 || exit 1
f=$(find $O/prof -name "*kernel_trace.csv" | head -1)
[ -n "$f" ] && python3 scripts/timeline.py "$f" conv1c_fwd > $O/timeline.txt && cat $O/timeline.txt
exit 0
