# Round 5: cost of the fused-statistics tail (DTFE_DIAG icr: 128 = records only, 64 = + ticket, 0 = + fold)
set -o pipefail
O=gpurun_out/r5imgstats2
mkdir -p $O
for d in 0 64 128; do
  echo "== icr=$d"
  DTFE_DIAG=icr=$d timeout -k 10 120 python3 bench/resnet20_kernels.py --only "conv2 fwd,bn_stats" > $O/k$d.txt 2>&1 || { tail -5 $O/k$d.txt; exit 1; }
  grep -v amdgpu.ids $O/k$d.txt
done
