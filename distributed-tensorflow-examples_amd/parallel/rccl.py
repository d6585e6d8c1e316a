"""Native RCCL communicator whose collectives are hipGraph-capturable.

``torch.distributed`` (ProcessGroupNCCL) issues each collective on an internal
stream guarded by a watchdog thread - fine for eager steps, but the framework's
data-parallel step is one hipGraph replay per step.  ``RcclComm`` owns a second,
private RCCL communicator over the same ranks (csrc/bindings/comm_ops.cpp:
ncclCommInitRank + ncclAllReduce on the caller's current stream), so the
gradient all-reduce becomes an ordinary graph node:

    compute stream:  ... fc wgrad -> cast bucket -> [fork] conv dgrad/wgrad ... [join] -> Adam
    side stream:                                  \\-> ncclAllReduce(bucket) --/

The unique id travels over the existing process group (rank 0 creates it).
Collectives must be issued in the same order on every rank - the step program
guarantees that; the first (eager) warm-up steps establish RCCL's peer
connections before any capture.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from .. import ops

SUM, MAX, MIN, AVG = 0, 1, 2, 3


class RcclComm:
    def __init__(self, device, group=None):
        ops.require()
        self.device = torch.device(device)
        self.group = group
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        lib = torch.ops.dtfe
        if self.rank == 0:
            uid = lib.rccl_unique_id()
        else:
            uid = torch.zeros(lib.rccl_id_bytes(), dtype=torch.uint8)
        if self.world > 1:
            box = [uid.numpy().tobytes()]
            src = dist.get_global_rank(group, 0) if group is not None else 0
            dist.broadcast_object_list(box, src=src, group=group, device=self.device)
            uid = torch.frombuffer(bytearray(box[0]), dtype=torch.uint8).clone()
        self.handle = lib.rccl_init(uid, self.world, self.rank, self.device.index or 0)

    def all_reduce(self, t: torch.Tensor, op: int = SUM):
        """In-place all-reduce of ``t`` on the current stream (capturable)."""
        torch.ops.dtfe.rccl_all_reduce(t, self.handle, op)

    def broadcast(self, t: torch.Tensor, root: int = 0):
        torch.ops.dtfe.rccl_broadcast(t, root, self.handle)

    def status(self) -> int:
        """0 while healthy, else RCCL's asynchronous error code (ncclCommGetAsyncError; no device
        sync - safe to poll from a watchdog thread while the step graph is blocked)."""
        if self.handle is None:
            return 0
        return int(torch.ops.dtfe.rccl_status(self.handle))

    def abort(self):
        """ncclCommAbort: release collectives stuck on a dead peer; the process exits next."""
        if self.handle is not None:
            torch.ops.dtfe.rccl_abort(self.handle)
            self.handle = None

    def close(self):
        if self.handle is not None:
            torch.ops.dtfe.rccl_destroy(self.handle)
            self.handle = None
