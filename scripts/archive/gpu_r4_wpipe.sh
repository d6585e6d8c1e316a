# ResNet-50 weight-gradient k-tile ring (DTFE_IG_WPIPE) under the 192-workgroup target, alternating on one box; GPU tests first
set -o pipefail
O=gpurun_out/r4wp
mkdir -p $O
for r in 1 2 3; do
  for t in 1 2 0; do
    DTFE_IG_WPIPE=$t timeout -k 10 300 python3 bench.py --model resnet50 --steps 20 --warmup 5 > $O/r50_${t}_$r.log 2>&1 || { tail -5 $O/r50_${t}_$r.log; exit 1; }
    echo "wpipe=$t $(grep -o '"value": [0-9.]*' $O/r50_${t}_$r.log) $(grep -o '"ms_per_step": [0-9.]*' $O/r50_${t}_$r.log)"
  done
done
