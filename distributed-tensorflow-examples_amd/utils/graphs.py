"""hipGraph capture of a whole training step.

A step program in this framework is a fixed sequence of kernel launches over
pre-allocated buffers (no allocation, no host sync), so it can be captured
once into a hipGraph (``torch.cuda.CUDAGraph`` is hipGraph on ROCm) and
replayed: one host call per step instead of ~15 kernel launches.  This is the
MI355X replacement for TF's graph executor on the per-step hot path.
"""
from __future__ import annotations

import os

import torch


def graphs_enabled(default: bool = True) -> bool:
    v = os.environ.get("DTFE_GRAPHS")
    if v is None:
        return default
    return v not in ("0", "false", "no")


class StepGraph:
    """Capture ``fn`` (no args) into a hipGraph after ``warmup`` eager runs."""

    def __init__(self, fn, warmup: int = 2, enabled: bool = True, pool=None, capture_error_mode: str = "global"):
        """capture_error_mode "thread_local": only this thread's capture-unsafe HIP calls
        invalidate the capture (other threads - e.g. the c10d watchdog - may keep polling
        their own events while a step with an in-graph RCCL all-reduce is recorded)."""
        self.fn = fn
        self.capture_error_mode = capture_error_mode
        self.warmup = warmup
        self.enabled = enabled and torch.cuda.is_available()
        self.graph = None
        self.pool = pool
        self._calls = 0
        self.capture_error = None

    def __call__(self):
        if not self.enabled:
            return self.fn()
        if self.graph is not None:
            self.graph.replay()
            return None
        self._calls += 1
        if self._calls <= self.warmup:
            return self.fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        try:
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                with torch.cuda.graph(g, pool=self.pool, stream=s, capture_error_mode=self.capture_error_mode):
                    self.fn()
            torch.cuda.current_stream().wait_stream(s)
            self.graph = g
            # the capture itself did not execute the step: replay it once now
            self.graph.replay()
        except Exception as e:  # noqa: BLE001 - fall back to eager launches, keep the reason
            self.capture_error = e
            self.enabled = False
            torch.cuda.synchronize()
            self.fn()
        return None


class MultiStepGraph:
    """``steps`` training steps per hipGraph replay (TF2's ``steps_per_execution``): a captured step ends
    with its optimizer launch and the next replay's first launch waits for the host's next graph launch -
    between replays the GPU idles for the graph-launch latency (~5 us after a 190 us CNN step, 8-18 us
    after the reference's 60-200 us GAN / autoencoder / LSTM steps in the kernel traces).  Captured
    back to back, consecutive steps are ordinary stream-ordered launches.  Every step is still a full
    training step (device-side sampling, forward, backward, all-reduce, optimizer); ``run(n)`` executes
    exactly n of them: whole S-step replays, then single-step replays for the remainder."""

    def __init__(self, fn, steps: int = 1, warmup: int = 2, enabled: bool = True,
                 capture_error_mode: str = "global", finish=None):
        """``finish``: called after the last step of every replay (and of every eager block) - e.g. the
        CNN trainer's join_side(), which rejoins a side stream once per replay instead of once per step."""
        self.steps = max(1, int(steps))

        def one():
            fn()
            if finish is not None:
                finish()
        self.one = StepGraph(one, warmup=warmup, enabled=enabled, capture_error_mode=capture_error_mode)

        def many():
            for _ in range(self.steps):
                fn()
            if finish is not None:
                finish()
        self.many = (StepGraph(many, warmup=1, enabled=enabled, capture_error_mode=capture_error_mode)
                     if self.steps > 1 else None)

    @property
    def graph(self):
        return self.one.graph if self.many is None else self.many.graph

    @property
    def capture_error(self):
        return self.one.capture_error or (self.many.capture_error if self.many is not None else None)

    def __call__(self):
        self.one()

    def prime(self) -> int:
        """Run steps until both graphs (S-step and single-step) are captured - so no capture falls inside a
        timed region; returns the number of (real, training) steps run."""
        n = 0
        for g, k in ((self.many, self.steps), (self.one, 1)):
            while g is not None and g.enabled and g.graph is None:
                g()
                n += k
        return n

    def run(self, n: int):
        while self.many is not None and n >= self.steps:
            self.many()
            n -= self.steps
        for _ in range(n):
            self.one()
