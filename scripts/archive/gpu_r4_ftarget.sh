# ResNet-50 forward / stride-1 data-gradient split-K target sweep, alternating on one box; GPU tests first
set -o pipefail
O=gpurun_out/r4ft
mkdir -p $O
for r in 1 2 3; do
  for t in 200 120 320; do
    AB_FTARGET=$t timeout -k 10 300 python3 bench.py --model resnet50 --steps 20 --warmup 5 > $O/r50_${t}_$r.log 2>&1 || { tail -5 $O/r50_${t}_$r.log; exit 1; }
    echo "ftarget=$t $(grep -o '"value": [0-9.]*' $O/r50_${t}_$r.log) $(grep -o '"ms_per_step": [0-9.]*' $O/r50_${t}_$r.log)"
  done
done
