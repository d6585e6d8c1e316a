"""MNIST conv2 weight gradient (persistent kernel + partial-sum reduce) time vs batch and grid cap.
python bench/conv2w_scale.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dtfe  # noqa: E402,F401
from dtfe import ops  # noqa: E402
from conv2_scale import timeit  # noqa: E402

dev, bf = "cuda", torch.bfloat16
for B in (256, 1024, 4096):
    p1 = torch.randn(B, 14, 14, 32, device=dev).to(bf)
    dp = torch.randn(B, 7, 7, 64, device=dev).to(bf)
    am = torch.randint(0, 4, (B, 7, 7, 64), device=dev, dtype=torch.uint8)
    dw = torch.zeros(64, 5, 5, 32, device=dev)
    db = torch.zeros(64, device=dev)
    ws = torch.empty(ops.wgrad_ws_floats(64, 800), device=dev)
    kw = dict(B=B, SH=14, SW=14, CS=32, OH=14, OW=14, N=64, KH=5, KW=5, stride=1, pad=2)
    row = []
    for mb in (0, 128):
        t = timeit(lambda: ops.imgwgrad(p1, dw, db, dy_pooled=dp, dy_argmax=am, workspace=ws, max_blocks=mb, **kw))
        row.append("blocks<=%s %7.1f us (%6.1f TF)" % (mb or 256, t, 2.0 * B * 196 * 64 * 800 / t / 1e6))
    print("B=%5d  " % B + "   ".join(row), flush=True)
