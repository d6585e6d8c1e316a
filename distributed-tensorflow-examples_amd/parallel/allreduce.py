"""Bucketed gradient all-reduce over RCCL (BASELINE.json "ring all-reduce mode").

Gradients live in one flat fp32 buffer ordered by backward completion, so a
bucket is a contiguous slice.  ``launch(i)`` is called from the step program
the moment bucket i's last gradient kernel has been *enqueued*: the RCCL
all-reduce is issued asynchronously (ProcessGroupNCCL runs it on its own HIP
stream, ordered after the producer kernels by an event), so it overlaps the
backward kernels that follow on the compute stream.  ``wait()`` joins the
compute stream to every outstanding bucket before the optimizer.

Programs that report backward progress call ``ready(lo)`` (every gradient at flat
offset >= lo is final; buckets are ordered back to front, the order backward
produces them) and ``flush()`` launches whatever is left.

With ``comm`` (a ``parallel.rccl.RcclComm``) the buckets go through dtfe's own RCCL
communicator on a side HIP stream forked from the compute stream instead of
ProcessGroupNCCL: every launch / join is a plain stream operation, so a whole
data-parallel step - backward, overlapped all-reduce, optimizer - can be captured
into one hipGraph (bench.py, train.py at world > 1).

Optionally the wire format is bf16 (half the xGMI bytes): a cast kernel packs
the bucket into a bf16 shadow buffer, the all-reduce runs on it, and the fused
optimizer consumes the bf16 sums directly (``grad16``) with 1/world folded in.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from .. import ops


class BucketAllReduce:
    def __init__(self, flat_grad: torch.Tensor, buckets, group=None, comm_dtype=torch.float32, comm=None):
        self.flat = flat_grad
        self.comm = comm
        self.side = torch.cuda.Stream(device=flat_grad.device) if comm is not None else None
        self._forked = False
        self.buckets = list(buckets)
        self.group = group
        self.comm_dtype = comm_dtype
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.shadow = None
        if comm_dtype == torch.bfloat16:
            self.shadow = torch.empty(flat_grad.numel(), dtype=torch.bfloat16, device=flat_grad.device)
        self._works = []
        self._work_of = {}
        self._done_ev = [torch.cuda.Event() for _ in self.buckets] if comm is not None else []
        self._next = 0  # next bucket (in launch order) not yet launched this step

    @property
    def grad16(self):
        return self.shadow

    def launch(self, i: int, after=None):
        """Start bucket i's all-reduce.  ``after``: extra hipEvents its gradients depend on beyond
        the current stream's work so far (e.g. weight gradients computed on another stream)."""
        lo, hi = self.buckets[i]
        if self.comm is not None:
            # fork: the side stream waits for everything enqueued so far (the bucket's producers)
            # plus the given events; the cast to the wire dtype runs on the side stream too, so
            # the compute stream never waits for a producer on a third stream
            self.side.wait_stream(torch.cuda.current_stream(self.flat.device))
            for ev in after or ():
                self.side.wait_event(ev)
            with torch.cuda.stream(self.side):
                buf = self._pack(lo, hi)
                self.comm.all_reduce(buf)
                self._done_ev[i].record(self.side)
            self._forked = True
            return
        for ev in after or ():
            torch.cuda.current_stream(self.flat.device).wait_event(ev)
        buf = self._pack(lo, hi)
        if self.world == 1:
            return
        self._works.append(dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=self.group, async_op=True))
        self._work_of[i] = self._works[-1]

    def _pack(self, lo: int, hi: int):
        if self.shadow is not None:
            ops.cast_(self.flat[lo:hi], self.shadow[lo:hi])
            return self.shadow[lo:hi]
        return self.flat[lo:hi]

    def wait_bucket(self, i: int):
        """Make the current stream wait for bucket i's all-reduce only (later buckets may still
        be in flight)."""
        if self.comm is not None:
            torch.cuda.current_stream(self.flat.device).wait_event(self._done_ev[i])
        elif i in self._work_of:
            self._work_of[i].wait()

    def ready(self, lo: int, after=None):
        """Backward progress hook: every gradient at flat offset >= lo is final (once the
        current stream's work so far and the events ``after`` complete).  Launches the buckets
        (in order) that lie entirely above lo, so their all-reduce overlaps the rest of the
        backward pass."""
        while self._next < len(self.buckets) and self.buckets[self._next][0] >= lo:
            self.launch(self._next, after)
            self._next += 1

    def flush(self):
        """Launch every bucket the backward hooks have not."""
        while self._next < len(self.buckets):
            self.launch(self._next)
            self._next += 1

    def wait_launched(self):
        """Make the current stream wait for every bucket launched so far (the step goes on;
        ``wait()`` still closes the step)."""
        if self._forked:
            torch.cuda.current_stream(self.flat.device).wait_stream(self.side)
        for w in self._works:
            w.wait()

    def wait(self):
        if self._forked:  # join the side stream back into the compute stream
            torch.cuda.current_stream(self.flat.device).wait_stream(self.side)
            self._forked = False
        for w in self._works:
            w.wait()
        self._works.clear()
        self._work_of.clear()
        self._next = 0
