#!/usr/bin/env python
"""fc1 data / weight gradient GEMMs (B=1024) on one tile id, replayed N times - a short workload for
rocprofv3 --pmc passes (scripts/pmc.sh).   python bench/fc_probe.py --tile 22 --reps 20"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dtfe  # noqa: E402,F401
from dtfe import ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--tile", type=int, default=22)
ap.add_argument("--reps", type=int, default=20)
ap.add_argument("--which", default="dgrad,wgrad")
a = ap.parse_args()
B, K1, FC = 1024, 3136, 1024
d, bf = "cuda", torch.bfloat16
p2 = torch.randn(B, K1, device=d).to(bf)
w1 = (torch.randn(FC, K1, device=d) * 0.02).to(bf)
dz = torch.randn(B, FC, device=d).to(bf)
dp2 = torch.empty(B, K1, device=d, dtype=bf)
gw = torch.zeros(FC, K1, device=d)
gb = torch.zeros(FC, device=d)
for _ in range(a.reps):
    if "dgrad" in a.which:
        ops.gemm(dz, w1, dp2, M=B, N=K1, K=FC, bmode=ops.RMAJ, ldb=K1, aux=p2, aux_act=ops.ACT_RELU, tile=a.tile)
    if "wgrad" in a.which:
        ops.gemm(dz, p2, gw, M=FC, N=K1 + 1, K=B, amode=ops.RMAJ, lda=FC, bmode=ops.RMAJ, ldb=K1, ldc=K1,
                 b_ones_row=K1, bias_out=gb, tile=a.tile)
torch.cuda.synchronize()
print("ok")
