"""Per-phase step timers ("hipEvent-based per-phase timers behind a flag",
"optionally emit a chrome trace").

``PhaseTimer(device)``: ``with t.phase("comm"): ...`` records a pair of hipEvents
around the phase on the current stream (GPU) or wall-clock on CPU; ``summary()``
synchronizes once and returns {phase: ms} for the last step.  The events are
recorded on the stream, so kernels queued asynchronously are measured where they
actually run, not where the host enqueued them.

With ``trace_path`` every phase of every step is also kept as a Chrome trace-event
("X" complete event, microseconds since the timer was created, one ``tid`` per rank) and
``close()`` writes the JSON array - open it in chrome://tracing or Perfetto.
"""
from __future__ import annotations

import contextlib
import json
import time

import torch


class PhaseTimer:
    def __init__(self, device, trace_path: str | None = None, rank: int = 0):
        self.gpu = torch.device(device).type == "cuda"
        self._marks = []
        self.trace_path = trace_path
        self.rank = rank
        self.events = []
        self._t0_wall = time.perf_counter()
        self._t0 = None
        if self.gpu:
            self._t0 = torch.cuda.Event(enable_timing=True)
            self._t0.record()

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
            if self.trace_path:
                start_ms = self._t0.elapsed_time(a) if self.gpu else (a - self._t0_wall) * 1000.0
                self.events.append({"name": name, "ph": "X", "ts": round(start_ms * 1000.0, 3),
                                    "dur": round(ms * 1000.0, 3), "pid": 0, "tid": self.rank,
                                    "cat": "gpu" if self.gpu else "cpu"})
        self._marks = []
        return out

    def close(self):
        """Write the collected trace events (no-op without ``trace_path``)."""
        if self._marks:
            self.summary()
        if self.trace_path:
            with open(self.trace_path, "w") as f:
                json.dump({"traceEvents": self.events, "displayTimeUnit": "ms"}, f)

    @staticmethod
    def format(d):
        return "phases: " + " ".join("%s %.3fms" % (k, v) for k, v in d.items())
