# ResNet-50: wgrad slab cap (AB_WPARTMB) and BN statistics grid cap scale (AB_SCAP / 4), alternating on one box
set -o pipefail
O=gpurun_out/r4misc
mkdir -p $O
for r in 1 2 3; do
  for v in 32:4 16:4 64:4 32:2 32:8; do
    m=${v%%:*}; c=${v##*:}
    AB_WPARTMB=$m AB_SCAP=$c timeout -k 10 300 python3 bench.py --model resnet50 --steps 20 --warmup 5 > $O/r50_${m}_${c}_$r.log 2>&1 || { tail -5 $O/r50_${m}_${c}_$r.log; exit 1; }
    echo "part_mb=$m scap=$c/4 $(grep -o '"ms_per_step": [0-9.]*' $O/r50_${m}_${c}_$r.log)"
  done
done
