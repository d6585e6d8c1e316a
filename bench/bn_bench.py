"""Per-shape timing of the BatchNorm HIP kernels on the ResNet-50 (batch 64) activation shapes:
microseconds per launch and effective HBM bandwidth (bytes the kernel must move / time).

    python bench/bn_bench.py [--batch 64]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import dtfe  # noqa: E402,F401
from dtfe import ops  # noqa: E402

SHAPES = [(112, 64), (56, 64), (56, 256), (56, 128), (28, 128), (28, 512), (28, 256), (14, 256), (14, 1024),
          (14, 512), (7, 512), (7, 2048)]


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1000 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    args = ap.parse_args()
    dev = "cuda"
    print(f"{'HxW':>6} {'C':>5} {'MB':>7} | {'stats':>14} {'apply':>14} {'bwd_stats':>14} {'bwd_apply':>14} "
          f"{'bwd_stats(x)':>14} {'bwd_apply(x)':>14}")
    for hw, C in SHAPES:
        shape = (args.batch, hw, hw, C)
        x = torch.randn(*shape, device=dev).to(torch.bfloat16)
        dy = torch.randn(*shape, device=dev).to(torch.bfloat16)
        y = torch.empty_like(x)
        dx = torch.empty_like(x)
        st, st2 = torch.zeros(2 * C, device=dev), torch.zeros(2 * C, device=dev)
        mean, inv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
        gamma, beta = torch.ones(C, device=dev), torch.zeros(C, device=dev)
        nb = x.numel() * 2
        ops.bn_stats(x, st)
        res = []
        for fn, nbytes in (
            (lambda: ops.bn_stats(x, st), nb),
            (lambda: ops.bn_apply(x, st, gamma, beta, y, mean=mean, invstd=inv), 2 * nb),
            (lambda: ops.bn_bwd_stats(dy, y, x, mean, inv, st2), 3 * nb),
            (lambda: ops.bn_bwd_apply(dy, y, x, mean, inv, gamma, st2, dx), 4 * nb),
            (lambda: ops.bn_bwd_stats(dy, None, x, mean, inv, st2, gamma=gamma, beta=beta), 2 * nb),
            (lambda: ops.bn_bwd_apply(dy, None, x, mean, inv, gamma, st2, dx, beta=beta), 3 * nb),
        ):
            us = timeit(fn)
            res.append(f"{us:6.1f}us {nbytes / us / 1e6:5.2f}TB")
        print(f"{hw:>3}x{hw:<3} {C:>5} {nb / 1e6:7.1f} | " + " ".join(f"{r:>14}" for r in res), flush=True)


if __name__ == "__main__":
    main()
