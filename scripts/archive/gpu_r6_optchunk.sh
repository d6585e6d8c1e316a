#!/bin/bash
# Round 6: optimizer work-item size A/B (DTFE_OPT_CHUNK) on the small-model steps and ResNet-20.
set -o pipefail
O=gpurun_out/r6oc; mkdir -p $O
for r in 1 2; do for c in 8192 2048 1024; do
  echo "chunk=$c" >> $O/ab.txt
  DTFE_OPT_CHUNK=$c timeout -k 10 120 python bench/ref_models.py --steps 400 --warmup 40 >> $O/ab.txt 2>&1 || exit 1
  DTFE_OPT_CHUNK=$c timeout -k 10 200 python bench.py --model resnet20 --steps 20 --warmup 5 2>/dev/null | tail -1 >> $O/ab.txt || exit 1
done; done
grep -v amdgpu.ids $O/ab.txt | sed 's/"config".*//'
