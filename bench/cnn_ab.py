#!/usr/bin/env python
"""MNIST-CNN bench step A/B of MnistCnnTrainer attributes, alternating in one process (same box, same
build): each arm is "name=value[,name=value]" applied to every trainer right after construction.
    python bench/cnn_ab.py --arms "side_adam=1" "side_adam=0" [--rounds 2] [--prewarm_ms 150]"""
import argparse
import contextlib
import importlib
import io
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import dtfe  # noqa: E402,F401
from dtfe.models import mnist_cnn  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--arms", nargs="+", required=True)
ap.add_argument("--rounds", type=int, default=2)
ap.add_argument("--prewarm_ms", type=float, default=150.0)
ap.add_argument("--steps", type=int, default=20)
args = ap.parse_args()

_init = mnist_cnn.MnistCnnTrainer.__init__
_arm = {}


def _patched(self, *a, **kw):
    for k, v in _arm.items():  # "module.NAME=v": a module constant of dtfe.<module>, set before construction
        if "." in k:
            mod, name = k.rsplit(".", 1)
            m = importlib.import_module("dtfe." + mod)
            setattr(m, name, type(getattr(m, name))(int(v)) if isinstance(getattr(m, name), bool) else
                    type(getattr(m, name))(v))
    _init(self, *a, **kw)
    for k, v in _arm.items():
        if "." in k:
            continue
        setattr(self, k, type(getattr(self, k))(v) if not isinstance(getattr(self, k), bool) else bool(int(v)))


mnist_cnn.MnistCnnTrainer.__init__ = _patched
for r in range(args.rounds):
    for arm in args.arms:
        _arm.clear()
        _arm.update(kv.split("=") for kv in arm.split(",") if kv)
        out = io.StringIO()
        with contextlib.redirect_stdout(out):
            bench.main(["--steps", str(args.steps), "--warmup", "5", "--prewarm_ms", str(args.prewarm_ms)])
        line = [ln for ln in out.getvalue().splitlines() if ln.startswith("{")][-1]
        print("%-28s %.4f ms/step" % (arm, json.loads(line)["ms_per_step"]), flush=True)
