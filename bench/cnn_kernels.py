#!/usr/bin/env python
"""Per-kernel timing of the MNIST-CNN step program (hipEvent-timed, interleaved rounds).

    python bench/cnn_kernels.py --batch_size 1024 --iters 50

Each op of MnistCnnTrainer.forward_backward()/apply() is replayed in isolation
on the trainer's own buffers; reports median/min microseconds per op and the
achieved TFLOP/s for the GEMM-shaped ones.
"""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dtfe  # noqa: E402,F401
from dtfe import ops  # noqa: E402
from dtfe.models.mnist_cnn import C1, C2, FC, KS, NCLS, MnistCnnTrainer  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch_size", type=int, default=1024)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--only", default="", help="comma-separated op names (default: all)")
    a = ap.parse_args()
    B = a.batch_size
    t = MnistCnnTrainer(B, "cuda")
    t.step()
    torch.cuda.synchronize()
    K1 = 7 * 7 * C2
    conv2_flops = 2.0 * B * 196 * C2 * KS * KS * C1
    fc1_flops = 2.0 * B * K1 * FC
    opsd = {
        "gather": (lambda: ops.gather_rows(t.data.images, t.x.view(B, -1), None, t.data.labels, t.labels, seed=1,
                                           counter=t.data_ctr, done=t.data_done), 0),
        "conv1_fwd": (lambda: ops.imgconv(t.w["wc1"], t.p1, src=t.x, bias=t.b["bc1"], argmax=t.a1,
                                          act=ops.ACT_RELU, pool=True, **t.ic1), 2.0 * B * 784 * 32 * 25),
        "conv2_fwd": (lambda: ops.imgconv(t.w["wc2"], t.p2, src=t.p1, bias=t.b["bc2"], argmax=t.a2,
                                          act=ops.ACT_RELU, pool=True, **t.ic2), conv2_flops),
        "fc1_fwd": (lambda: ops.gemm(t.p2, t.w["wd1"], t.h, M=B, N=FC, K=K1, bias=t.b["bd1"], act=ops.ACT_RELU,
                                     keep=t.keep, seed=2, counter=t.data_ctr), fc1_flops),
        "head": (lambda: ops.head_xent(t.h, t.w["out"], t.b["bout"], t.labels, t.dzf, t.dl, t.loss_sum,
                                       t.correct, None, scale=1.0 / B, inv_keep=1.0 / t.keep), 0),
        "head_noacc": (lambda: ops.head_xent(t.h, t.w["out"], t.b["bout"], t.labels, t.dzf, t.dl, None, None, None,
                                             scale=1.0 / B, inv_keep=1.0 / t.keep), 0),
        "head_wgrad": (lambda: ops.gemm(t.dl, t.h, t.gw["out"], M=NCLS, N=FC + 1, K=B, amode=ops.RMAJ, lda=16,
                                        bmode=ops.RMAJ, ldb=FC, ldc=FC, b_ones_row=FC, bias_out=t.gw["bout"],
                                        atomic=True, splits=max(1, min(16, B // 128)), tile=4), 0),
        "head_wgrad_k": (lambda: ops.head_wgrad(t.dl, t.h, t.gw["out"], t.gw["bout"], NCLS), 0),
        "fc1_dgrad": (lambda: ops.gemm(t.dzf, t.w["wd1"], t.dp2, M=B, N=K1, K=FC, bmode=ops.RMAJ, ldb=K1,
                                       aux=t.p2, aux_act=ops.ACT_RELU), fc1_flops),
        "fc1_wgrad": (lambda: ops.gemm(t.dzf, t.p2, t.gw["wd1"], M=FC, N=K1 + 1, K=B, amode=ops.RMAJ, lda=FC,
                                       bmode=ops.RMAJ, ldb=K1, ldc=K1, b_ones_row=K1, bias_out=t.gw["bd1"]),
                      fc1_flops),
        "conv2_dgrad": (lambda: ops.imgconv(t.wt["wc2"], t.dp1, src_pooled=t.dp2, src_argmax=t.a2,
                                            relu_mask=t.p1, flip_taps=True, **t.ic2_dgrad), conv2_flops),
        "conv2_wgrad": (lambda: ops.imgwgrad(t.p1, t.gw["wc2"], t.gw["bc2"], dy_pooled=t.dp2, dy_argmax=t.a2,
                                             **t.ic2), conv2_flops),
        "conv2_wgrad_ws": (lambda: ops.imgwgrad(t.p1, t.gw["wc2"], t.gw["bc2"], dy_pooled=t.dp2, dy_argmax=t.a2,
                                                workspace=t.ws_c2, max_blocks=t.c2_blocks, **t.ic2), conv2_flops),
        "conv1_wgrad": (lambda: ops.imgwgrad(t.x, t.gw["wc1"], t.gw["bc1"], dy_pooled=t.dp1, dy_argmax=t.a1,
                                             **t.ic1), 2.0 * B * 784 * 32 * 25),
        "adam": (lambda: t.opt.step(), 0),
        "grad_zero": (lambda: t.P.grad.zero_(), 0),
    }
    if a.only:
        opsd = {k: v for k, v in opsd.items() if k in a.only.split(",")}
    times = {k: [] for k in opsd}
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for _ in range(a.iters):
        for k, (fn, _) in opsd.items():
            ev[0].record()
            for _ in range(10):  # back-to-back launches: one launch on an idle GPU also times the host
                fn()
            ev[1].record()
            ev[1].synchronize()
            times[k].append(ev[0].elapsed_time(ev[1]) * 100)
    total = 0.0
    print("%-12s %10s %10s %10s" % ("op", "median_us", "min_us", "TFLOP/s"))
    for k, (fn, fl) in opsd.items():
        med, mn = statistics.median(times[k]), min(times[k])
        total += med
        tf = fl / (mn * 1e-6) / 1e12 if fl else float("nan")
        print("%-12s %10.1f %10.1f %10.1f" % (k, med, mn, tf))
    print("%-12s %10.1f" % ("sum", total))


if __name__ == "__main__":
    main()
