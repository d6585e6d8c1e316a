"""Per-launch floor of a captured hipGraph chain on one MI355X: N back-to-back launches of a
trivial kernel vs launches that touch a few MB (fill / copy), replayed and timed per launch.
Tells what a fused launch saves on the small-kernel ResNet-20 step (profiles/r5_launch_floor.txt)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from dtfe import ops  # noqa: E402


def per_launch_us(fn, n=200, reps=20):
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(n):
            fn()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps / n * 1e6


def main():
    d = torch.device("cuda")
    tiny = torch.empty(64, device=d)
    rows = [("fill 64 floats", lambda: tiny.fill_(1.0), 0)]
    for mb in (1, 4, 8, 32):
        n = mb * (1 << 20) // 4
        a, b = torch.empty(n, device=d), torch.empty(n, device=d)
        rows.append((f"fill {mb} MB", (lambda a=a: a.fill_(2.0)), mb))
        rows.append((f"copy {mb} MB", (lambda a=a, b=b: b.copy_(a)), 2 * mb))
    # this framework's small ResNet-20 kernels (stage 1: B=256, 32x32x16 bf16 = 8 MB)
    B, H, C = 256, 32, 16
    x = torch.randn(B, H, H, C, device=d).bfloat16()
    y, g = torch.empty_like(x), torch.randn_like(x)
    st = torch.zeros(2 * C, device=d)
    gam, bet = torch.ones(C, device=d), torch.zeros(C, device=d)
    mean, inv, mm, mv = (torch.zeros(C, device=d) for _ in range(4))
    f32 = torch.randn(B, 64, device=d)
    b16 = torch.empty(B, 64, device=d, dtype=torch.bfloat16)
    db = torch.zeros(64, device=d)
    rows += [("dtfe cast 16K", lambda: ops.cast_(f32, b16), 0),
             ("dtfe colsum", lambda: ops.colsum(f32, B, 64, 64, db), 0),
             ("dtfe bn_stats 8MB", lambda: ops.bn_stats(x, st), 8),
             ("dtfe bn_apply 8MB", lambda: ops.bn_apply(x, st, gam, bet, y, mean=mean, invstd=inv, moving_mean=mm,
                                                        moving_var=mv), 16),
             ("dtfe shortcut 8MB", lambda: ops.shortcut_grad_add(g, y, 1), 24)]
    print(f"{'launch':16s} {'us/launch':>10s} {'GB/s':>8s}")
    for name, fn, mb in rows:
        us = per_launch_us(fn)
        print(f"{name:16s} {us:10.2f} {mb * 1.048576e6 / us / 1e3 if mb else 0:8.0f}")
        sys.stdout.flush()


if __name__ == "__main__":
    main()
