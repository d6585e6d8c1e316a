#!/usr/bin/env python
"""Dense GEMM sweep on the MNIST-CNN fc shapes: our MFMA kernel per (tile, splits)
vs torch.mm (hipBLASLt) on the same operands.  hipEvent-timed, median of --iters.

    python bench/gemm_sweep.py --iters 30
"""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dtfe  # noqa: E402,F401
from dtfe import ops  # noqa: E402


def timeit(fn, iters, batch=10):
    """median over `iters` rounds of `batch` back-to-back launches (a single launch between two
    events on an idle GPU would also time the host's launch latency)"""
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        ev[0].record()
        for _ in range(batch):
            fn()
        ev[1].record()
        ev[1].synchronize()
        ts.append(ev[0].elapsed_time(ev[1]) * 1000 / batch)
    return statistics.median(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--tiles", type=lambda v: [int(t) for t in v.split(",")], default=[0, 2, 5, 6, 8, 10, 12],
                    help="tile ids (ops.TILE_DIMS)")
    ap.add_argument("--splits", type=lambda v: [int(t) for t in v.split(",")], default=None,
                    help="split-K factors for every tile (default 1,2,4 below tile 14, 1 above)")
    a = ap.parse_args()
    B, K1, FC = a.batch, 3136, 1024
    d, bf = "cuda", torch.bfloat16
    p2 = torch.randn(B, K1, device=d).to(bf)
    w1 = torch.randn(FC, K1, device=d).to(bf) * 0.02
    dz = torch.randn(B, FC, device=d).to(bf)
    h = torch.empty(B, FC, device=d, dtype=bf)
    dp2 = torch.empty(B, K1, device=d, dtype=bf)
    gw = torch.zeros(FC, K1, device=d)
    gb = torch.zeros(FC, device=d)
    bias = torch.zeros(FC, device=d)
    shapes = {
        # name: (fn(tile, splits), torch reference fn, flops)
        "fc1_fwd": (lambda t, s: ops.gemm(p2, w1, h, M=B, N=FC, K=K1, bias=bias, act=ops.ACT_RELU, tile=t, splits=s),
                    lambda: torch.mm(p2, w1.t()), 2.0 * B * FC * K1),
        "fc1_dgrad": (lambda t, s: ops.gemm(dz, w1, dp2, M=B, N=K1, K=FC, bmode=ops.RMAJ, ldb=K1, aux=p2,
                                            aux_act=ops.ACT_RELU, tile=t, splits=s),
                      lambda: torch.mm(dz, w1), 2.0 * B * FC * K1),
        "fc1_wgrad": (lambda t, s: ops.gemm(dz, p2, gw, M=FC, N=K1 + 1, K=B, amode=ops.RMAJ, lda=FC, bmode=ops.RMAJ,
                                            ldb=K1, ldc=K1, b_ones_row=K1, bias_out=gb, tile=t, splits=s,
                                            atomic=s > 1 and t < 5),
                      lambda: torch.mm(dz.t(), p2), 2.0 * B * FC * K1),
    }
    for name, (fn, ref, fl) in shapes.items():
        tr = timeit(ref, a.iters)
        print(f"{name:10s} torch.mm {tr:8.1f} us {fl / tr / 1e6:7.1f} TFLOP/s", flush=True)
        for tile in a.tiles:
            row = []
            for s in (a.splits or ((1, 2, 4) if tile < 14 else (1,))):
                try:
                    t = timeit(lambda: fn(tile, s), a.iters)
                except RuntimeError:
                    row.append(f"s{s}:      n/a        ")
                    continue
                row.append(f"s{s}:{t:7.1f}us/{fl / t / 1e6:6.1f}TF")
            bm, bn = ops.TILE_DIMS[tile]
            print(f"{name:10s} {bm:3d}x{bn:<3d}{'g' if tile >= 5 else ' '}{tile:<3d} " + "  ".join(row), flush=True)


if __name__ == "__main__":
    main()
