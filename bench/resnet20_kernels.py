#!/usr/bin/env python
"""Per-launch timing of the ResNet-20 (B=256) step's kernels, each replayed N times inside one
captured hipGraph (so the numbers include the in-graph launch floor, ~1.6 us - bench/launch_floor.py).

    python bench/resnet20_kernels.py [--only conv,bn,...] [--wgrad_grids 256,128,64]

Blocks timed: s1 = stage 1 (16 ch, 32x32), s2 = stage 2 (32 ch, 16x16), s2d = its stride-2 entry
block, s3 = stage 3 (64 ch, 8x8).  Rows: conv fwd, BN statistics / apply, BN backward statistics /
apply, conv data / weight gradient (+ partial reduce), shortcut gradient."""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dtfe  # noqa: E402,F401
from dtfe import ops  # noqa: E402
from dtfe.models.resnet import ResNetModel  # noqa: E402


NO_GRAPH = False


def per_launch_us(fn, n=40, reps=10):
    if NO_GRAPH:  # (PMC collection: plain launches)
        for _ in range(n):
            fn()
        torch.cuda.synchronize()
        return 0.0
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        for _ in range(2):
            fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(n):
            fn()
    g.replay()
    torch.cuda.synchronize()
    best = 1e30
    for _ in range(3):
        t = time.perf_counter()
        for _ in range(reps):
            g.replay()
        torch.cuda.synchronize()
        best = min(best, (time.perf_counter() - t) / reps / n * 1e6)
    return best


def bwd_stats(bn, dy, x):
    xx, y, mean, inv, gam, beta, st, act = bn.bwd_stats_args(x)
    ops.bn_bwd_stats(dy, y, xx, mean, inv, st, act, gamma=gam, beta=beta)


def phases(prog, blocks):
    """Phase boundaries of the persistent conv (imgconv_persist_kernel stamps): 0 start, 1 weights
    staged + LDS zeroed, 2 first image in LDS, 3 first tile pass's MFMAs done, 4 epilogue into LDS
    done, 5 copy-out issued, 6 workgroup end - microseconds after the earliest workgroup start."""
    lib = ops.require()
    names = ["start", "w+zero", "img", "mfma1", "epi", "store", "end"]
    print("conv              " + " ".join(f"{n:>14s}" for n in names))
    for tag, i in (("s1", 1), ("s2", 4), ("s3", 7)):
        b = blocks[i]
        for kind in ("fwd", "dgrad"):
            c = b.conv2
            ts = torch.zeros(256 * 8, dtype=torch.int64, device="cuda")
            if kind == "fwd":
                g = c.ic
                call = lambda: lib.imgconv(b.bn1.y, None, None, c.w, None, c.y, None, None, g["B"], g["SH"], g["SW"],
                                           g["CS"], g["OH"], g["OW"], g["N"], g["KH"], g["KW"], g["stride"], g["pad"],
                                           False, ops.ACT_NONE, False, 1, None, 1, ts)
            else:
                call = lambda: lib.imgconv(b.dc2, None, None, c.wt, None, b.dh1, None, None, c.B, c.OH, c.OW, c.cout,
                                           c.H, c.W, c.cin, c.k, c.k, 1, c.k - 1 - c.pad, True, ops.ACT_NONE, False,
                                           c.dil, None, 1, ts)
            for _ in range(5):
                call()
            torch.cuda.synchronize()
            t = ts.view(256, 8)[:, :7].double().cpu()
            t0 = t[:, 0].min()
            rel = (t - t0) / 100.0  # 100 MHz -> us
            med = rel.median(0).values
            mx = rel.max(0).values
            print(f"{tag} conv2 {kind:6s}  " + " ".join(f"{m:6.2f}/{x:6.2f} " for m, x in zip(med, mx)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch_size", type=int, default=256)
    ap.add_argument("--wgrad_grids", default="")
    ap.add_argument("--only", default="", help="comma-separated substrings of the rows to time")
    ap.add_argument("--phases", action="store_true",
                    help="per-workgroup phase stamps of the whole-image conv (s_memrealtime, 10 ns ticks)")
    ap.add_argument("--no_graph", action="store_true", help="plain launches (for rocprofv3 --pmc passes)")
    a = ap.parse_args()
    global NO_GRAPH
    NO_GRAPH = a.no_graph
    prog = ResNetModel(arch="resnet20").program(torch.device("cuda"), a.batch_size)
    prog.compute_grads()
    torch.cuda.synchronize()
    blocks = prog.L["blocks"]
    st = prog.L["stem"]
    dn, P = prog.L["dense"], prog.P
    rows = [("stem fwd", lambda: st.fwd(prog.x)), ("stem wgrad", lambda: st.wgrad(prog.dc_stem, prog.x)),
            ("dense head", lambda: ops.dense_head(prog.feat16, P.view(dn.kernel), P.view(dn.bias), prog.y, prog.logits,
                                                  prog.loss, prog.correct, P.gview(dn.kernel), P.gview(dn.bias),
                                                  prog.dfeat16, 1.0 / a.batch_size))]
    for tag, i in (("s1", 1), ("s2d", 3), ("s2", 4), ("s3", 7)):
        b = blocks[i]
        dout = prog.d_in[i + 1]
        dx = prog.d_in[i]
        rows += [
            (f"{tag} conv1 fwd", lambda b=b: b.conv1.fwd(b.x)),
            (f"{tag} conv2 fwd", lambda b=b: b.conv2.fwd(b.bn1.y)),
            (f"{tag} bn_stats", lambda b=b: ops.bn_stats(b.conv2.y, b.bn2.stats)),
            (f"{tag} bn1 apply", lambda b=b: b.bn1.fwd((b.conv1.y, True))),
            (f"{tag} bn2 apply+res", lambda b=b: b.bn2.fwd((b.conv2.y, True), res=b.x, rstride=b.stride)),
            (f"{tag} bn2 bwd_stats", lambda b=b, d=dout: bwd_stats(b.bn2, d, b.conv2.y)),
            (f"{tag} bn2 bwd_apply", lambda b=b, d=dout: b.bn2.bwd(d, b.conv2.y, b.dc2, dres=b.dres,
                                                                   stats_done=True)),
            (f"{tag} bn1 bwd (2 passes)", lambda b=b: b.bn1.bwd(b.dh1, b.conv1.y, b.dc1)),
            (f"{tag} conv2 wgrad+reduce", lambda b=b: b.conv2.wgrad(b.dc2, b.bn1.y)),
            (f"{tag} conv1 wgrad+reduce", lambda b=b: b.conv1.wgrad(b.dc1, b.x)),
            (f"{tag} conv2 dgrad", lambda b=b: b.conv2.dgrad(b.dc2, b.dh1)),
            (f"{tag} conv1 dgrad", lambda b=b, dx=dx: b.conv1.dgrad(b.dc1, dx)),
            (f"{tag} shortcut add", lambda b=b, dx=dx: ops.shortcut_grad_add(b.dres, dx, b.stride)),
        ]
        for gcap in [int(x) for x in a.wgrad_grids.split(",") if x]:
            c = b.conv2
            rows.append((f"{tag} conv2 wgrad grid {gcap}",
                         lambda c=c, b=b, gcap=gcap: ops.imgwgrad(b.bn1.y, c.gw, None, dy=b.dc2, max_blocks=gcap,
                                                                  **c.ic)))
    print(f"{'launch':30s} {'us':>8s}")
    if a.phases:
        phases(prog, blocks)
        return
    only = [x for x in a.only.split(",") if x]
    for name, fn in rows:
        if only and not any(o in name for o in only):
            continue
        print(f"{name:30s} {per_launch_us(fn):8.2f}")
        sys.stdout.flush()


if __name__ == "__main__":
    main()
