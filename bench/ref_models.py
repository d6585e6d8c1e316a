#!/usr/bin/env python
"""Per-step time of the reference's three workloads on one MI355X.

The reference's only performance output is the per-step ``AvgTime: %3.2fms`` print
(gan/distributed_gan.py:196, encoder/distributed_encoder.py:167, lstm/distributed_lstm.py:130)
around batch fetch + ``sess.run`` of one training step.  This times the same step - stage
the batch (on-device copy), forward, backward, the TF1 optimizer(s) and the global step -
captured into one hipGraph, on synthetic MNIST-shaped data with the reference batch sizes
and hyper-parameters.

    python bench/ref_models.py [--models gan,encoder,lstm] [--steps 200] [--warmup 20]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import dtfe  # noqa: E402,F401
from dtfe.optim import Optimizer  # noqa: E402
from dtfe.train import MODELS  # noqa: E402
from dtfe.utils.graphs import MultiStepGraph  # noqa: E402


def time_model(name, steps, warmup, graph=True, steps_per_graph=1):
    cls, lr = MODELS[name]
    model = cls(lr=lr)
    dev = torch.device("cuda", 0)
    B = model.default_batch
    prog = model.program(dev, B, seed=0)
    gstep = torch.zeros(1, dtype=torch.int32, device=dev)
    opts = [Optimizer(cfg, prog.P, var_list=vl, global_step=gstep, beta_power_names=bp)
            for cfg, vl, bp in model.opt_groups]
    g = torch.Generator().manual_seed(1)
    x = torch.rand(B, 784, generator=g).to(dev)
    y = torch.nn.functional.one_hot(torch.randint(0, 10, (B,), generator=g), 10).float().to(dev)

    def step():
        prog.load_batch((x, y))
        prog.compute_grads()
        # all of the step's optimizers in one launch (TF: the minimize ops of one sess.run)
        Optimizer.step_all(opts, [model.gs_increments if i == len(opts) - 1 else 0 for i in range(len(opts))])

    run = MultiStepGraph(step, steps_per_graph, warmup=2, enabled=graph)
    run.run(warmup)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run.run(steps)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / steps * 1e3
    return {"model": name, "batch": B, "ms_per_step": round(ms, 4), "hip_graph": run.graph is not None,
            "steps_per_graph": run.steps, "global_step": int(gstep.item())}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", default="gan,encoder,lstm")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--no_graph", action="store_true")
    ap.add_argument("--steps_per_graph", type=int, default=1, help="training steps per hipGraph replay")
    a = ap.parse_args()
    for m in a.models.split(","):
        print(json.dumps(time_model(m, a.steps, a.warmup, graph=not a.no_graph, steps_per_graph=a.steps_per_graph)),
              flush=True)


if __name__ == "__main__":
    main()
