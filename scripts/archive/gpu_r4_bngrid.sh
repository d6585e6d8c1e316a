# Round-4: BN statistics grid cap A/B (DTFE_BN_SGRID) on the ResNet-50 B=256 shapes + ResNet-50 step
set -o pipefail
O=gpurun_out/r4bngrid
mkdir -p $O
for g in 512 256 128; do
  DTFE_BN_SGRID=$g timeout -k 10 200 python3 bench/bn_bench.py --batch 256 > $O/bn_$g.txt 2>&1 || { tail -5 $O/bn_$g.txt; exit 1; }
  echo "== cap $g"; grep -v amdgpu.ids $O/bn_$g.txt | awk '{print $1, $2, $5, $9, $13}'
done
for r in 1 2; do
  for g in 512 256 128; do
    DTFE_BN_SGRID=$g timeout -k 10 300 python3 bench.py --model resnet50 --steps 20 --warmup 5 > $O/r50_${g}_$r.log 2>&1 || { tail -5 $O/r50_${g}_$r.log; exit 1; }
    echo "r50 cap=$g $(grep -o '"value": [0-9.]*' $O/r50_${g}_$r.log) $(grep -o '"ms_per_step": [0-9.]*' $O/r50_${g}_$r.log)"
  done
done
