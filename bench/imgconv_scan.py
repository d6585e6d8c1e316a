#!/usr/bin/env python
"""Time the whole-image conv kernels vs batch size: slope = per-image cost,
intercept = prologue (weight staging) + launch.  MNIST conv2 fwd / dgrad / wgrad."""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dtfe  # noqa: E402,F401
from dtfe import ops  # noqa: E402


def t(fn, iters=30):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        ev[0].record()
        fn()
        ev[1].record()
        ev[1].synchronize()
        ts.append(ev[0].elapsed_time(ev[1]) * 1000)
    return statistics.median(ts)


bf = torch.bfloat16
for B in (256, 512, 1024, 2048, 4096):
    x = torch.randn(B, 14, 14, 32, device="cuda").to(bf)
    w = torch.randn(64, 5, 5, 32, device="cuda").to(bf)
    wt = torch.randn(32, 5, 5, 64, device="cuda").to(bf)
    bias = torch.zeros(64, device="cuda")
    y = torch.empty(B, 7, 7, 64, device="cuda", dtype=bf)
    am = torch.empty(B, 7, 7, 64, device="cuda", dtype=torch.uint8)
    dp1 = torch.empty(B, 14, 14, 32, device="cuda", dtype=bf)
    dw = torch.zeros(64, 5, 5, 32, device="cuda")
    db = torch.zeros(64, device="cuda")
    g = dict(B=B, SH=14, SW=14, CS=32, OH=14, OW=14, N=64, KH=5, KW=5, stride=1, pad=2)
    gd = dict(B=B, SH=14, SW=14, CS=64, OH=14, OW=14, N=32, KH=5, KW=5, stride=1, pad=2)
    f = t(lambda: ops.imgconv(w, y, src=x, bias=bias, argmax=am, act=ops.ACT_RELU, pool=True, **g))
    d = t(lambda: ops.imgconv(wt, dp1, src_pooled=y, src_argmax=am, relu_mask=x, flip_taps=True, **gd))
    wg = t(lambda: ops.imgwgrad(x, dw, db, dy_pooled=y, dy_argmax=am, **g))
    print(f"B={B:5d} fwd {f:7.1f} us  dgrad {d:7.1f} us  wgrad {wg:7.1f} us", flush=True)
