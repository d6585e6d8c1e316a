#!/bin/bash
# Round 6: small-GEMM waves per tile by grid size (default policy) vs 16 everywhere (gs=16) vs 4 everywhere.
set -o pipefail
O=gpurun_out/r6gs4; mkdir -p $O
for r in 1 2 3; do for cfg in none gs=1 gs=2 gs=3; do
  echo "$cfg" >> $O/ab.txt
  DTFE_DIAG=$cfg timeout -k 10 120 python bench/ref_models.py --models gan,encoder --steps 400 --warmup 40 >> $O/ab.txt 2>&1 || exit 1
done; done
grep -v amdgpu.ids $O/ab.txt
