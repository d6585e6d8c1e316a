#!/bin/bash
# Round 6: small-GEMM waves per tile (K split) x operand chunk A/B on the GAN and autoencoder steps.
set -o pipefail
O=gpurun_out/r6gs2; mkdir -p $O
for r in 1 2; do for cfg in gs=4 gs=4,gc=8 gs=8,gc=8 gs=16 gs=16,gc=4 gs=8,gc=4; do
  echo "$cfg" >> $O/ab.txt
  DTFE_DIAG=$cfg timeout -k 10 120 python bench/ref_models.py --models gan,encoder --steps 400 --warmup 40 >> $O/ab.txt 2>&1 || exit 1
done; done
grep -v amdgpu.ids $O/ab.txt
