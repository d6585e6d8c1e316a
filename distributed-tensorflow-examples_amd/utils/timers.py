"""Per-phase step timers ("hipEvent-based per-phase timers behind a flag").

``PhaseTimer(device)``: ``with t.phase("comm"): ...`` records a pair of hipEvents
around the phase on the current stream (GPU) or wall-clock on CPU; ``summary()``
synchronizes once and returns {phase: ms} for the last step.  The events are
recorded on the stream, so kernels queued asynchronously are measured where they
actually run, not where the host enqueued them.
"""
from __future__ import annotations

import contextlib
import time

import torch


class PhaseTimer:
    def __init__(self, device):
        self.gpu = torch.device(device).type == "cuda"
        self._marks = []

    @contextlib.contextmanager
    def phase(self, name):
        if self.gpu:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            yield
            b.record()
            self._marks.append((name, a, b))
        else:
            t0 = time.perf_counter()
            yield
            self._marks.append((name, t0, time.perf_counter()))

    def summary(self):
        out = {}
        if self.gpu and self._marks:
            self._marks[-1][2].synchronize()
        for name, a, b in self._marks:
            ms = a.elapsed_time(b) if self.gpu else (b - a) * 1000.0
            out[name] = out.get(name, 0.0) + ms
        self._marks = []
        return out

    @staticmethod
    def format(d):
        return "phases: " + " ".join("%s %.3fms" % (k, v) for k, v in d.items())
