#!/usr/bin/env python
"""Where the ps's apply time goes: the MNIST CNN's fused Adam reading its bf16 gradient from an
uncached hipIpc mailbox (hipDeviceMallocUncached, the ps data plane's allocation) vs from ordinary
cached device memory, and the bulk copy out of the uncached buffer.  One process, one GPU.

    python bench/ps_mailbox.py [--iters 50]
"""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dtfe  # noqa: E402,F401
from dtfe import ops  # noqa: E402
from dtfe.models.mnist_cnn import MnistCnnTrainer  # noqa: E402


class _Raw:
    """__cuda_array_interface__ over a raw device pointer (torch.as_tensor aliases it)."""

    def __init__(self, ptr, n, typestr):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": typestr, "data": (ptr, False), "version": 3}


def timeit(fn, iters, batch=10):
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
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    lib = ops.require()
    tr = MnistCnnTrainer(1024, dev, seed=1)
    n = tr.P.master.numel()
    h = lib.ps_ipc_alloc(n * 2 + 4096, 0)
    ptr = lib.ps_ipc_ptr(h)
    # int16 view (bf16 has no typestr); reinterpret as bf16
    uc = torch.as_tensor(_Raw(ptr, n, "<i2"), device=dev).view(torch.bfloat16)
    cached = torch.randn(n, device=dev).to(torch.bfloat16) * 1e-3
    uc.copy_(cached)
    torch.cuda.synchronize()
    t_uc = timeit(lambda: tr.opt.step(grad16=uc, gscale=1.0, gs_inc=0), a.iters)
    t_c = timeit(lambda: tr.opt.step(grad16=cached, gscale=1.0, gs_inc=0), a.iters)
    dst = torch.empty_like(cached)
    t_cp_uc = timeit(lambda: dst.copy_(uc), a.iters)
    t_cp_c = timeit(lambda: dst.copy_(cached), a.iters)
    t_wr_uc = timeit(lambda: uc.copy_(cached), a.iters)
    mb = n * 2 / 1e6
    print("params %d (bf16 gradient %.1f MB)" % (n, mb))
    print("fused Adam, gradient in uncached IPC memory : %6.1f us" % t_uc)
    print("fused Adam, gradient in cached device memory: %6.1f us" % t_c)
    print("copy uncached -> cached : %6.1f us (%.0f GB/s)" % (t_cp_uc, mb * 1e3 / t_cp_uc))
    print("copy cached -> cached   : %6.1f us (%.0f GB/s)" % (t_cp_c, mb * 1e3 / t_cp_c))
    print("copy cached -> uncached : %6.1f us (%.0f GB/s)" % (t_wr_uc, mb * 1e3 / t_wr_uc))
    del uc
    torch.cuda.synchronize()
    lib.ps_ipc_close(h)


if __name__ == "__main__":
    main()
