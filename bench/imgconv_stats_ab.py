#!/usr/bin/env python
"""ResNet-20 whole-image forward convs (B=256) with / without the fused output BN statistics, and the
bn_stats pass they replace.  DTFE_DIAG icr=<bits> ablates parts of the fused path (1024: no
workgroup reduction / hand-off, 256: reduction + partial row only, 512: + ticket, no final fold).
    DTFE_DIAG=icr=256 python bench/imgconv_stats_ab.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dtfe  # noqa: E402,F401
from dtfe import ops  # noqa: E402


def timeit(fn, reps=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000 / reps


B = 256
print("DTFE_DIAG=%s" % os.environ.get("DTFE_DIAG", ""))
print("%-22s %9s %9s %9s" % ("conv", "plain us", "+stats us", "bn_stats"))
for H, CI, N, s in ((32, 16, 16, 1), (32, 16, 32, 2), (16, 32, 32, 1), (16, 32, 64, 2), (8, 64, 64, 1)):
    x = torch.randn(B, H, H, CI, device="cuda").to(torch.bfloat16)
    w = (torch.randn(N, 3, 3, CI, device="cuda") * 0.1).to(torch.bfloat16)
    OH = H // s
    kw = dict(B=B, SH=H, SW=H, CS=CI, OH=OH, OW=OH, N=N, KH=3, KW=3, stride=s, pad=1)
    y = torch.empty(B, OH, OH, N, device="cuda", dtype=torch.bfloat16)
    st = torch.zeros(2 * N, device="cuda")
    t0 = timeit(lambda: ops.imgconv(w, y, src=x, **kw))
    t1 = timeit(lambda: ops.imgconv(w, y, src=x, stats=st, **kw))
    t2 = timeit(lambda: ops.bn_stats(y, st))
    print("%-22s %9.2f %9.2f %9.2f" % ("%dx%dx%d->%d s%d" % (H, H, CI, N, s), t0, t1, t2))
