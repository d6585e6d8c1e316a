# Round 6 (session 2): ResNet-50 56x56 1x1 convs under each implicit-GEMM tile (DTFE_IG_TILE)
set -o pipefail
O=gpurun_out/${1:-r6s2i}
mkdir -p $O
for t in auto 128x64 64x64; do
  if [ $t = auto ]; then unset DTFE_IG_TILE; else export DTFE_IG_TILE=$t; fi
  timeout -k 10 120 python3 bench/write_roofline.py --reps 20 > $O/roof_$t.log 2>&1 || { tail -5 $O/roof_$t.log; exit 1; }
  echo "== tile $t"; grep conv $O/roof_$t.log
done
