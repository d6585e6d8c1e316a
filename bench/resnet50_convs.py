#!/usr/bin/env python
"""Per-layer timing of the ResNet-50 convolutions (fwd / dgrad / wgrad) through
dtfe's conv ops, next to stock PyTorch (MIOpen, channels_last bf16) on the same
shapes.  One line per distinct layer shape: us and TFLOP/s for each pass.

    python bench/resnet50_convs.py [--batch 64] [--reps 20] [--no-torch]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import dtfe  # noqa: E402,F401
from dtfe import ops  # noqa: E402


def shapes():
    """(H, C, Cout, k, stride) of every distinct ResNet-50 conv with its multiplicity."""
    out = {}
    H, cin = 56, 64
    for stage, (w, n) in enumerate(((64, 3), (128, 4), (256, 6), (512, 3))):
        for i in range(n):
            s = 2 if (stage and i == 0) else 1
            convs = [(H, cin, w, 1, 1), (H, w, w, 3, s), (H // s, w, 4 * w, 1, 1)]
            if i == 0:
                convs.append((H, cin, 4 * w, 1, s))
            for c in convs:
                out[c] = out.get(c, 0) + 1
            H, cin = H // s, 4 * w
    return out


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
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--no-torch", action="store_true")
    ap.add_argument("--only", default="", help="H,C,Cout,k,s[;...]: just these layers (PMC runs)")
    a = ap.parse_args()
    only = {tuple(int(v) for v in t.split(",")) for t in a.only.split(";") if t}
    B, dev = a.batch, "cuda"
    tot = {"ours": [0.0, 0.0, 0.0], "torch": [0.0, 0.0, 0.0]}
    print("%-28s %4s | %22s | %22s | %22s" % ("layer (H C->Cout kxk /s)", "n", "fwd us (TF/s)", "dgrad us (TF/s)",
                                              "wgrad us (TF/s)"))
    for (H, C, Cout, k, s), n in shapes().items():
        if only and (H, C, Cout, k, s) not in only:
            continue
        pad = (k - 1) // 2
        OH = (H + 2 * pad - k) // s + 1
        g = dict(B=B, H=H, W=H, C=C, Cout=Cout, OH=OH, OW=OH, KH=k, KW=k, stride=s, pad=pad)
        fl = 2.0 * B * OH * OH * Cout * k * k * C
        x = torch.randn(B, H, H, C, device=dev).to(torch.bfloat16)
        w = (torch.randn(Cout, k, k, C, device=dev) * 0.05).to(torch.bfloat16)
        wt = w.permute(3, 1, 2, 0).contiguous()
        dy = torch.randn(B, OH, OH, Cout, device=dev).to(torch.bfloat16)
        y = torch.empty(B, OH, OH, Cout, device=dev, dtype=torch.bfloat16)
        dx = torch.empty(B, H, H, C, device=dev, dtype=torch.bfloat16)
        dw = torch.zeros(Cout, k, k, C, device=dev)
        t = [timeit(lambda: ops.conv_fwd(x, w, None, y, None, g, act=ops.ACT_NONE), a.reps),
             timeit(lambda: ops.conv_dgrad(dy, wt, dx, g), a.reps),
             timeit(lambda: ops.conv_wgrad(dy, x, dw, None, g, 1.0), a.reps)]
        line = "%-28s %4d | " % ("%d %d->%d %dx%d /%d" % (H, C, Cout, k, k, s), n)
        line += " | ".join("%9.1f (%7.1f)" % (u, fl / u * 1e-6) for u in t)
        for i in range(3):
            tot["ours"][i] += n * t[i]
        if not a.no_torch:
            xn = x.permute(0, 3, 1, 2)  # channels_last views
            wn = w.permute(0, 3, 1, 2)
            dyn = dy.permute(0, 3, 1, 2)
            tt = [timeit(lambda: F.conv2d(xn, wn, stride=s, padding=pad), a.reps),
                  timeit(lambda: torch.ops.aten.convolution_backward(dyn, xn, wn, None, (s, s), (pad, pad), (1, 1),
                                                                     False, (0, 0), 1, (True, False, False)), a.reps),
                  timeit(lambda: torch.ops.aten.convolution_backward(dyn, xn, wn, None, (s, s), (pad, pad), (1, 1),
                                                                     False, (0, 0), 1, (False, True, False)), a.reps)]
            line += "  || torch " + " ".join("%7.1f" % u for u in tt)
            if k == 1 and s == 1:  # a 1x1 conv is a plain GEMM: hipBLASLt via torch.mm for the bar
                a2, w2 = x.view(-1, C), w.view(Cout, C)
                line += "  || mm %7.1f (%7.1f)" % ((lambda u: (u, fl / u * 1e-6))(timeit(lambda: torch.mm(a2, w2.t()), a.reps)))
            for i in range(3):
                tot["torch"][i] += n * tt[i]
        print(line, flush=True)
    print("per-step conv totals (us): ours fwd %.0f dgrad %.0f wgrad %.0f = %.0f" %
          (*tot["ours"], sum(tot["ours"])))
    if not a.no_torch:
        print("                          torch fwd %.0f dgrad %.0f wgrad %.0f = %.0f" %
              (*tot["torch"], sum(tot["torch"])))


if __name__ == "__main__":
    main()
