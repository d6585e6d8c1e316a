# Round 5: BN statistics grid sweep on the ResNet-20 shapes + the shape-rule wgrad grid
set -o pipefail
O=gpurun_out/r5bngrid
mkdir -p $O
for g in 128 256 512 1024; do
  echo "== stats grid cap $g"
  DTFE_BN_SGRID=$g timeout -k 10 120 python3 bench/resnet20_kernels.py --only bn_stats,bwd_stats,bn1 > $O/g$g.txt 2>&1 || { tail -5 $O/g$g.txt; exit 1; }
  grep -v amdgpu.ids $O/g$g.txt
done
timeout -k 10 120 python3 bench/resnet20_kernels.py --only wgrad > $O/wgrad.txt 2>&1 || { tail -5 $O/wgrad.txt; exit 1; }
grep -v amdgpu.ids $O/wgrad.txt
