#!/usr/bin/env python
"""Isolated time of the one-launch dense classifier head at the LSTM shape (fp32, B=128, F=128, [F][NC] W)
and ResNet-20's (bf16, B=256, F=64), with DTFE_DIAG dh=<bits> phase ablations (1 logits, 2 softmax, 4 dW,
8 dfeat, 16 db, 32 feature staging).   python bench/dense_head_probe.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dtfe  # noqa: E402,F401
from dtfe import ops  # noqa: E402


def timeit(fn, reps=200):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000 / reps


d = "cuda"
cases = {}
for name, B, F, f32, wfm in (("lstm", 128, 128, True, True), ("resnet20", 256, 64, False, False)):
    NC = 10
    feat = torch.randn(B, F, device=d)
    feat = feat if f32 else feat.bfloat16()
    w = torch.randn(F, NC, device=d) if wfm else torch.randn(NC, F, device=d)
    b = torch.randn(NC, device=d)
    y = torch.nn.functional.one_hot(torch.randint(0, NC, (B,), device=d), NC).float()
    lg, loss, hits = torch.empty(B, NC, device=d), torch.zeros(1, device=d), torch.zeros(1, dtype=torch.int32, device=d)
    dw, db, df = torch.zeros_like(w), torch.zeros(NC, device=d), torch.empty_like(feat)
    cases[name] = lambda feat=feat, w=w, b=b, y=y, lg=lg, loss=loss, hits=hits, dw=dw, db=db, df=df, B=B, wfm=wfm: \
        ops.dense_head(feat, w, b, y, lg, loss, hits, dw, db, df, 1.0 / B, w_fmajor=wfm, store=wfm)
for bits in (0, 1, 2, 4, 8, 16, 32, 63):
    os.environ["DTFE_DIAG"] = "dh=%d" % bits
    print("dh=%-3d " % bits + "  ".join("%s %.2f us" % (k, timeit(f)) for k, f in cases.items()), flush=True)
