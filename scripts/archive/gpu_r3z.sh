# conv2 data gradient captured first: conv2 weight-gradient grid sweep (DTFE_CNN_C2_BLOCKS) vs default.
set -o pipefail
O=gpurun_out/r3z2
mkdir -p $O
for r in 1 2 3; do
  for v in d 160 176 192 208 224; do
    if [ $v = d ]; then unset DTFE_CNN_DGRAD_FIRST DTFE_CNN_C2_BLOCKS; else export DTFE_CNN_DGRAD_FIRST=1 DTFE_CNN_C2_BLOCKS=$v; fi
    timeout -k 10 120 python3 bench.py > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
    echo "$v $(grep -o '"ms_per_step": [0-9.]*' $O/b.log)"
  done
done
export DTFE_CNN_DGRAD_FIRST=1 DTFE_CNN_C2_BLOCKS=192
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 30 --warmup 5 > $O/prof.log 2>&1 || exit 1
f=$(find $O/prof -name "*kernel_trace.csv" | head -1)
[ -n "$f" ] && python3 scripts/timeline.py "$f" conv1c_fwd > $O/timeline.txt && cat $O/timeline.txt
exit 0
