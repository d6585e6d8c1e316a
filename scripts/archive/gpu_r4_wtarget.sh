# ResNet-50 weight-gradient split target sweep (workgroups per launch; slab cap MB), alternating on one box
set -o pipefail
O=gpurun_out/r4wt
mkdir -p $O
for r in 1 2 3; do
  for v in 512:32 192:32 160:32 224:32; do
    t=${v%%:*}; m=${v##*:}
    AB_WTARGET=$t AB_WPARTMB=$m timeout -k 10 300 python3 bench.py --model resnet50 --steps 20 --warmup 5 > $O/r50_${t}_${m}_$r.log 2>&1 || { tail -5 $O/r50_${t}_${m}_$r.log; exit 1; }
    echo "target=$t part_mb=$m $(grep -o '"value": [0-9.]*' $O/r50_${t}_${m}_$r.log) $(grep -o '"ms_per_step": [0-9.]*' $O/r50_${t}_${m}_$r.log)"
  done
done
