# Round 5: ablation of the runtime-geometry persistent conv on the ResNet-20 shapes
# (DTFE_DIAG icr=<bits>: 1 no epilogue stores, 2 no image staging, 4 no MFMA loop, 8 no weight loads)
set -o pipefail
O=gpurun_out/r5icr
mkdir -p $O
for d in 0 1 2 4 8 5 7 15; do
  echo "== icr=$d"
  DTFE_DIAG=icr=$d timeout -k 10 120 python3 bench/resnet20_kernels.py --only "conv1 fwd,conv2 dgrad" > $O/d$d.txt 2>&1 || { tail -5 $O/d$d.txt; exit 1; }
  grep -v amdgpu.ids $O/d$d.txt
done
