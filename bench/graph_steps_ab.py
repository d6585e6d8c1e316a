#!/usr/bin/env python
"""Steps per hipGraph replay: the MNIST CNN B=1024 training step captured 1, 2 or 4 times into one
graph, alternating rounds of 400 steps each (hipEvent-timed, one process).  Measures what the
graph-launch boundary between two replays costs per step.

    python bench/graph_steps_ab.py [--rounds 3] [--steps 400]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dtfe  # noqa: E402,F401
from dtfe.models.mnist_cnn import MnistCnnTrainer  # noqa: E402
from dtfe.utils.graphs import StepGraph  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=400)
    a = ap.parse_args()
    tr = MnistCnnTrainer(1024, torch.device("cuda", 0), seed=0)
    runners = {}
    for n in (1, 2, 4):
        def fn(n=n):
            for _ in range(n):
                tr.step()
        runners[n] = StepGraph(fn, warmup=1, capture_error_mode="thread_local")
        for _ in range(3):
            runners[n]()
        assert runners[n].graph is not None, runners[n].capture_error
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for _ in range(200):  # clocks up
        runners[1]()
    for r in range(a.rounds):
        for n, run in runners.items():
            torch.cuda.synchronize()
            ev[0].record()
            for _ in range(a.steps // n):
                run()
            ev[1].record()
            ev[1].synchronize()
            print("round %d  %d step(s) per replay: %.4f ms/step" % (r, n, ev[0].elapsed_time(ev[1]) / a.steps), flush=True)


if __name__ == "__main__":
    main()
