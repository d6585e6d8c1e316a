"""MNIST conv2 forward / data-gradient time vs batch (per-block fixed cost vs per-image cost of the
persistent whole-image kernels).  python bench/conv2_scale.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dtfe  # noqa: E402,F401
from dtfe import ops  # noqa: E402


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000 / reps


dev, bf = "cuda", torch.bfloat16
for B in (256, 512, 1024, 2048, 4096):
    x = torch.randn(B, 14, 14, 32, device=dev).to(bf)
    w = (torch.randn(64, 5, 5, 32, device=dev) * 0.1).to(bf)
    bias = torch.zeros(64, device=dev)
    y = torch.empty(B, 7, 7, 64, device=dev, dtype=bf)
    am = torch.empty(B, 7, 7, 64, device=dev, dtype=torch.uint8)
    kw = dict(B=B, SH=14, SW=14, CS=32, OH=14, OW=14, N=64, KH=5, KW=5, stride=1, pad=2)
    tf = timeit(lambda: ops.imgconv(w, y, src=x, bias=bias, argmax=am, act=ops.ACT_RELU, pool=True, **kw))
    wt = (torch.randn(32, 5, 5, 64, device=dev) * 0.1).to(bf)
    mask = torch.randn(B, 14, 14, 32, device=dev).to(bf)
    dx = torch.empty(B, 14, 14, 32, device=dev, dtype=bf)
    kd = dict(B=B, SH=14, SW=14, CS=64, OH=14, OW=14, N=32, KH=5, KW=5, pad=2, flip_taps=True)
    td = timeit(lambda: ops.imgconv(wt, dx, src_pooled=y, src_argmax=am, relu_mask=mask, **kd))
    fl = 2.0 * B * 196 * 64 * 800
    print(f"B={B:5d}  fwd {tf:7.1f} us ({fl / tf / 1e6:6.1f} TF)   dgrad {td:7.1f} us ({fl / td / 1e6:6.1f} TF)", flush=True)
