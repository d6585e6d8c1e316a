# Round-4: ResNet-50 weight-gradient side stream priority A/B
set -o pipefail
O=gpurun_out/r4prio
mkdir -p $O
for r in 1 2; do
  for p in 0 -1; do
    DTFE_SIDE_PRIO=$p timeout -k 10 300 python3 bench.py --model resnet50 --steps 20 --warmup 5 > $O/r50_${p}_$r.log 2>&1 || { tail -5 $O/r50_${p}_$r.log; exit 1; }
    echo "prio=$p r$r $(grep -o '"value": [0-9.]*' $O/r50_${p}_$r.log) $(grep -o '"ms_per_step": [0-9.]*' $O/r50_${p}_$r.log)"
  done
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
DTFE_SIDE_PRIO=-1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 bench.py --model resnet50 --steps 6 --warmup 4 > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
f=$(find $O/prof -name "*kernel_trace.csv" | head -1); python3 scripts/timeline.py "$f" stem_fwd > $O/timeline.txt; tail -3 $O/timeline.txt
