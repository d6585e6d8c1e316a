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
