"""Gradient-collective selection for the data-parallel modes.

Two capturable all-reduce engines exist (both issue on the caller's current stream):

* ``RcclComm`` - dtfe's own RCCL communicator (ring / tree channels over xGMI);
* ``IpcComm``  - the one-launch hipIpc two-shot kernel reading the 7 peers directly.

``make_comm(mode="auto")`` builds both, self-checks the IPC path, then times each on the
actual bucket sizes of the job (max over ranks, so every rank takes the same decision)
and routes every bucket size to the faster engine.  An IPC failure of any kind degrades
to RCCL instead of failing the job.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from .ipc import IpcComm
from .rccl import RcclComm

# Gradient bucket size (MB of fp32 gradient; half that on a bf16 wire).  What was measured: ResNet-50
# B=256 data-parallel over the IPC engine at W=2 with BOTH ranks sharing one MI355X (the only multi-rank
# setup this pool allows; profiles/r4_comm_rehearsal.txt): 2 / 4 / 8 / 16 / 32 MB -> 55.5 / 54.9 / 53.9 /
# 54.1 / 53.6 ms per step, flat within 3.5 %.  What that can NOT show: the xGMI side - per-link
# bandwidth, the 7-peer fan-in of one IPC launch and RCCL's ring latency on a real node - so the choice
# below is reasoned, not measured on xGMI: 16 MB keeps ResNet-50's 51 MB bf16 gradient in 7 buckets so
# the first all-reduces start while the backward still has most of its layers to run (the overlap an
# 8-GPU node needs), at the IPC staging cap of one 8 MB bucket.  Override with --bucket_mb.
DEFAULT_BUCKET_MB = 16.0


class RoutedComm:
    """``all_reduce`` dispatching on the tensor's byte size (decided once, at setup)."""

    def __init__(self, default, routes=None, names=None, group=None, device=None):
        self.default = default
        self.routes = dict(routes or {})
        self.names = dict(names or {})
        self.comms = [default] + [c for c in self.routes.values() if c is not default]
        self.group = group
        self.device = device

    @property
    def world(self) -> int:
        """Ranks the collective engine spans (reported by bench.py as ranks_seen_by_comm)."""
        return int(self.default.world)

    def local_status(self) -> int:
        """Non-zero when an engine of THIS rank reported a failure: the IPC kernel's barrier-timeout
        word (reading it synchronizes the device) or RCCL's asynchronous error code."""
        bad = 0
        for c in self.comms:
            if hasattr(c, "status"):
                bad = max(bad, int(c.status()))
        return bad

    def check_health(self):
        """Raise on EVERY rank if any rank's engine failed since setup.

        The all-reduce runs inside replayed hipGraphs; a peer that misses an IPC barrier for longer
        than the timeout makes the kernel set its error word and leave the bucket half reduced, and
        an RCCL error only surfaces through ncclCommGetAsyncError - nothing else would notice.
        Callers do it every ``log_every`` steps and once at the end; the decision is agreed over the
        group so all ranks stop together instead of training on diverged replicas.  (A peer that
        died outright is the comm watchdog's job, parallel/health.py CommWatchdog: this agreement
        itself would need the dead peer.)"""
        bad = float(self.local_status())
        if _agree(bad, self.group, self.device) > 0:
            raise RuntimeError("all-reduce engine failure on %s rank: gradients of that step were not "
                               "fully reduced; replicas may have diverged" % ("this" if bad else "another"))

    def abort(self):
        """Release collectives blocked on a dead peer (ncclCommAbort; the IPC kernel ends on its own
        barrier timeout).  The process must exit afterwards."""
        for c in self.comms:
            if hasattr(c, "abort"):
                c.abort()

    def all_reduce(self, t: torch.Tensor, *args):
        self.routes.get(t.numel() * t.element_size(), self.default).all_reduce(t, *args)

    def describe(self) -> str:
        if not self.names:
            return type(self.default).__name__
        return ", ".join("%.2fMB:%s" % (b / 1e6, n) for b, n in sorted(self.names.items()))

    def close(self):
        for c in self.comms:
            c.close()


def _time_comm(comm, t, group, iters=8):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(3):
        comm.all_reduce(t)
    torch.cuda.synchronize()
    dist.barrier(group=group)
    s.record()
    for _ in range(iters):
        comm.all_reduce(t)
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def _cpu_ok(group):
    """True when the group can reduce a CPU tensor (gloo, or a cpu:gloo,cuda:nccl group)."""
    try:
        return "gloo" in str(dist.get_backend(group))
    except Exception:  # noqa: BLE001
        return False


def _agree(x: float, group, device) -> float:
    t = torch.tensor([x], dtype=torch.float64, device="cpu" if _cpu_ok(group) else device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())


def make_comm(device, group=None, bucket_bytes=(), dtype=torch.bfloat16, mode: str = "auto", log=None,
              timeout_s: float = 30.0):
    """Collective engine for buckets of the given byte sizes.  mode: rccl | ipc | auto.
    ``timeout_s``: the IPC kernel's barrier timeout (a peer that never arrives)."""
    device = torch.device(device)
    cap = max([int(b) for b in bucket_bytes] + [1 << 20]) + 4096
    if mode == "ipc":  # IPC only (no RCCL communicator: also works for several ranks sharing one GPU)
        ipc = IpcComm(device, group, cap_bytes=cap, timeout_s=timeout_s)
        return RoutedComm(ipc, {int(b): ipc for b in bucket_bytes}, {int(b): "ipc" for b in bucket_bytes},
                          group=group, device=device)
    rccl = RcclComm(device, group)
    if mode == "rccl":
        return RoutedComm(rccl, group=group, device=device)
    ipc = None
    try:
        ipc = IpcComm(device, group, cap_bytes=cap, timeout_s=timeout_s, fallback=rccl)
        ok = 1.0
    except Exception as e:  # noqa: BLE001 - any IPC trouble (mapping, self-check, timeout) -> RCCL
        ok = 0.0
        if log:
            log("ipc all-reduce unavailable (%s); using RCCL" % (e,))
    if _agree(1.0 - ok, group, device) > 0:   # one rank failed: nobody uses IPC
        if ipc is not None:
            ipc.close()
        return RoutedComm(rccl, group=group, device=device)
    routes, names = {}, {}
    esz = torch.tensor([], dtype=dtype).element_size()
    for b in sorted(set(int(x) for x in bucket_bytes)):
        t = torch.zeros(max(1, b // esz), dtype=dtype, device=device)
        t_r = _agree(_time_comm(rccl, t, group), group, device)
        t_i = _agree(_time_comm(ipc, t, group), group, device)
        routes[b] = ipc if t_i < t_r else rccl
        names[b] = "ipc" if t_i < t_r else "rccl"
        if log:
            log("all-reduce %.2f MB %s: rccl %.1f us, ipc %.1f us -> %s"
                % (b / 1e6, dtype, t_r * 1e3, t_i * 1e3, names[b]))
    if _agree(float(ipc.status()), group, device) != 0:   # a timing run tripped a barrier timeout somewhere
        ipc.close()
        return RoutedComm(rccl, group=group, device=device)
    return RoutedComm(rccl, routes, names, group=group, device=device)
