#!/usr/bin/env python
"""HBM write roofline next to ResNet-50's write-heavy 56x56 1x1 convolutions (B=256).

    python bench/write_roofline.py [--batch 256] [--reps 20]

Rows: a pure 411 MB bf16 fill, a 411 MB copy, a 103 MB -> 411 MB channel broadcast (the bytes of
the 64 -> 256 1x1 forward), and the implicit-GEMM 1x1 convs themselves (64 -> 256 forward, with and
without the fused BN statistics; 256 -> 64's data gradient, which writes the 256-channel tensor).
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import dtfe  # noqa: E402,F401
from dtfe import ops  # noqa: E402


def timeit(fn, reps):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    B, dev = a.batch, "cuda"
    x64 = torch.randn(B, 56, 56, 64, device=dev).to(torch.bfloat16)
    y256 = torch.empty(B, 56, 56, 256, device=dev, dtype=torch.bfloat16)
    z256 = torch.randn(B, 56, 56, 256, device=dev).to(torch.bfloat16)
    w = (torch.randn(256, 1, 1, 64, device=dev) * 0.1).to(torch.bfloat16)
    wt = (torch.randn(256, 1, 1, 64, device=dev) * 0.1).to(torch.bfloat16)  # [C=256][1][1][Cout=64]
    st = torch.zeros(512, device=dev)
    g = dict(B=B, H=56, W=56, C=64, Cout=256, OH=56, OW=56, KH=1, KW=1, stride=1, pad=0)
    gd = dict(B=B, H=56, W=56, C=256, Cout=64, OH=56, OW=56, KH=1, KW=1, stride=1, pad=0)
    mb = lambda t: t.numel() * t.element_size() / 1e6  # noqa: E731
    rows = [
        ("fill 411 MB bf16", lambda: y256.fill_(0), mb(y256)),
        ("copy 411 MB -> 411 MB", lambda: y256.copy_(z256), 2 * mb(y256)),
        ("broadcast 103 MB -> 411 MB (repeat 4x)", lambda: y256.view(B, 56, 56, 4, 64).copy_(x64.unsqueeze(3).expand(B, 56, 56, 4, 64)),
         mb(x64) + mb(y256)),
        ("conv 1x1 64->256 fwd", lambda: ops.conv_fwd(x64, w, None, y256, None, g, act=ops.ACT_NONE), mb(x64) + mb(y256)),
        ("conv 1x1 64->256 fwd + BN stats", lambda: (st.zero_(), ops.conv_fwd(x64, w, None, y256, None, g, act=ops.ACT_NONE, stats=st)),
         mb(x64) + mb(y256)),
        ("conv 1x1 256->64 dgrad (writes 256 ch)", lambda: ops.conv_dgrad(x64, wt, y256, gd), mb(x64) + mb(y256)),
    ]
    print("%-44s %9s %9s %7s" % ("op", "us", "MB", "TB/s"))
    for name, fn, m in rows:
        us = timeit(fn, a.reps)
        print("%-44s %9.1f %9.1f %7.2f" % (name, us, m, m / us), flush=True)


if __name__ == "__main__":
    main()
