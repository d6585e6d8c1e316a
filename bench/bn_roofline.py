#!/usr/bin/env python
"""BatchNorm roofline of one ResNet-50 training step (B=256 by default).

Records every BatchNorm-family launch the real step issues (ops.bn_* / pool3 BN kernels called by
models/resnet.py, with their real arguments), then replays each launch on its own and reports
microseconds, the bytes it must move (every activation-sized tensor argument is read or written
exactly once: x, residual, dy, y / ReLU bits, outputs) and the effective HBM bandwidth against the
≈6.3 TB/s a streaming copy reaches on MI355X (MI355X_MICROARCH.md).  Rows are grouped by kind and
shape; the last line is the per-step BN total.

    python bench/bn_roofline.py [--batch 256] [--reps 10]

The conv-epilogue statistics folds (bn_part_stage1/2, launched from the C++ conv ops) are not
Python calls and are not in this table; see the rocprof kernel tables in profiles/.
"""
import argparse
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import dtfe  # noqa: E402,F401
from dtfe import ops  # noqa: E402

KINDS = ["bn_stats", "bn_apply", "bn_bwd_stats", "bn_bwd_apply", "bn_relu_pool3", "pool3_bn_bwd", "bn_infer"]
ROOF_TBS = 6.3


def _tensors(v):
    if isinstance(v, torch.Tensor):
        yield v
    elif isinstance(v, (list, tuple)):
        for u in v:
            yield from _tensors(u)


def _bytes(args, kwargs, min_numel=1 << 15):
    seen, n = set(), 0
    for t in _tensors(list(args) + list(kwargs.values())):
        if t.numel() >= min_numel and t.data_ptr() not in seen:
            seen.add(t.data_ptr())
            n += t.numel() * t.element_size()
    return n


def _label(kind, args, kwargs):
    x = args[0]
    shape = "x".join(str(s) for s in x.shape[1:])
    tags = []
    if kind == "bn_apply":
        if kwargs.get("res") is not None:
            tags.append("res")
        if kwargs.get("res_bn") is not None:
            tags.append("res_bn")
        if kwargs.get("mask_out") is not None:
            tags.append("bits")
    if kind in ("bn_bwd_stats", "bn_bwd_apply"):
        y = args[1]
        tags.append("x-mask" if y is None else ("bits" if y.dtype == torch.uint8 else "y"))
        if kind == "bn_bwd_stats" and (kwargs.get("res_bn") is not None or (len(args) > 9 and args[9] is not None)):
            tags.append("res_bn")
        if kind == "bn_bwd_apply" and kwargs.get("dres") is not None:
            tags.append("dres")
    return "%s[%s]" % (kind, ",".join(tags)) if tags else kind, shape


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    from dtfe.models.resnet import ResNetModel

    dev = torch.device("cuda", 0)
    model = ResNetModel(arch="resnet50")
    prog = model.program(dev, batch_size=a.batch, seed=0)
    g = torch.Generator(device="cpu").manual_seed(0)
    x = torch.rand(a.batch, 224, 224, 3, generator=g)
    y = torch.randint(0, 1000, (a.batch, 1), generator=g)
    prog.load_batch((x.to(dev), y.to(dev)))
    prog.compute_grads()  # warm every workspace
    torch.cuda.synchronize()

    rec = []
    orig = {k: getattr(ops, k) for k in KINDS}

    def wrap(kind):
        def f(*args, **kwargs):
            rec.append((kind, args, kwargs))
            return orig[kind](*args, **kwargs)
        return f

    for k in KINDS:
        setattr(ops, k, wrap(k))
    try:
        prog.compute_grads()
    finally:
        for k in KINDS:
            setattr(ops, k, orig[k])
    torch.cuda.synchronize()

    rows = collections.OrderedDict()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for kind, args, kwargs in rec:
        fn = orig[kind]
        fn(*args, **kwargs)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(a.reps):
            fn(*args, **kwargs)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1000 / a.reps
        key = _label(kind, args, kwargs)
        r = rows.setdefault(key, [0, 0.0, 0])
        r[0] += 1
        r[1] += us
        r[2] += _bytes(args, kwargs)
    print("# ResNet-50 B=%d: every BatchNorm launch of one training step, replayed alone (%d reps each)" %
          (a.batch, a.reps))
    print("%-36s %-12s %3s | %9s %9s %8s %6s | %9s" % ("kind", "shape", "n", "us/call", "MB/call", "TB/s", "roof%",
                                                    "us/step"))
    tot_us = tot_b = 0.0
    for (kind, shape), (n, us, b) in rows.items():
        tbs = b / us / 1e6
        print("%-36s %-12s %3d | %9.1f %9.1f %8.2f %5.0f%% | %9.1f" % (kind, shape, n, us / n, b / n / 1e6, tbs,
                                                                        100 * tbs / ROOF_TBS, us))
        tot_us += us
        tot_b += b
    print("per-step BN launches: %d, %.1f us, %.0f MB moved, %.2f TB/s effective (roofline at %.1f TB/s: %.1f us)" %
          (sum(r[0] for r in rows.values()), tot_us, tot_b / 1e6, tot_b / tot_us / 1e6, ROOF_TBS,
           tot_b / ROOF_TBS / 1e6))


if __name__ == "__main__":
    main()
