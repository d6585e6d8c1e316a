"""hipIpc two-shot all-reduce over xGMI ("custom IPC all-reduce for small
and medium buckets").

Every rank allocates one uncached exchange buffer, exports its IPC handle, and maps every
peer's buffer (``hipIpcOpenMemHandle``); one kernel launch (csrc/kernels/ipc_allreduce.hip)
then stages, reduces its 1/W segment by reading the W-1 peers directly over their
point-to-point xGMI links, and gathers the other segments - no host involvement, no
RCCL proxy, capturable in a hipGraph like any kernel.  Same ``all_reduce(t)`` interface
as ``RcclComm`` so ``BucketAllReduce(comm=...)`` takes either; buckets larger than the
staging capacity go to ``fallback`` (an RcclComm) when one is given.

Construction runs a self-check (rank-dependent values, summed and compared on every
rank, plus the kernel's barrier-timeout flag); a mismatch or timeout raises, and
callers fall back to RCCL.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from .. import ops


# workgroups per all-reduce launch (the kernel's own cap is 128): its workgroups spin at the
# exchange barriers while the peers' halves arrive, holding CUs the overlapped backward kernels
# could use.  bench/ipc_interference.py, MNIST CNN fc bucket (6.5 MB bf16) beside conv2's backward,
# two ranks on ONE GPU (profiles/r5_ipc_grid_cap.txt): conv+all-reduce span 128 -> 217 / 205 us,
# 64 -> 214 / 181, 32 -> 229 / 237, 16 -> 175 / 175 (all-reduce alone 125 -> 150 us).  16 is the span
# minimum there.  On a node each GPU hosts one rank and reads its 7 peers over xGMI, whose per-link
# rate - not the workgroup count - bounds a 16-workgroup launch; that part is unmeasured here, so
# the cap applies only to buffers up to DEFAULT_CAP_UPTO (the CNN's 6.5 MB fc bucket and smaller,
# the ones that overlap a short backward); larger ones (ResNet-50's 16 MB buckets) keep the
# kernel's full 128-workgroup grid.
DEFAULT_MAX_BLOCKS = 16
DEFAULT_CAP_UPTO = 8 << 20


class IpcComm:
    def __init__(self, device, group=None, cap_bytes: int = 64 << 20, timeout_s: float = 30.0, fallback=None,
                 self_check: bool = True, max_blocks: int | None = None):
        ops.require()
        self.device = torch.device(device)
        self.group = group
        self.fallback = fallback
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.handle = None
        lib = torch.ops.dtfe
        # every step that can fail on one rank is followed by an all-rank agreement, so a
        # failure raises on EVERY rank at the same point (no rank is left in a collective)
        mine, err = b"", None
        try:
            self.handle = lib.ipc_create(int(cap_bytes), self.rank, self.world, self.device.index or 0,
                                         float(timeout_s))
            self.cap = lib.ipc_capacity(self.handle)
            lib.ipc_set_max_blocks(self.handle, int(max_blocks or DEFAULT_MAX_BLOCKS), DEFAULT_CAP_UPTO)
            mine = lib.ipc_handle(self.handle).numpy().tobytes()
        except Exception as e:  # noqa: BLE001
            err = e
        self._agree(err, "exchange buffer")
        allh = [mine]
        if self.world > 1:
            allh = [None] * self.world
            dist.all_gather_object(allh, mine, group=group)
        try:
            lib.ipc_open(self.handle, torch.stack([torch.frombuffer(bytearray(h), dtype=torch.uint8) for h in allh]))
        except Exception as e:  # noqa: BLE001
            err = e
        self._agree(err, "peer mapping")
        if self_check:
            try:
                self.check()
            except Exception as e:  # noqa: BLE001
                err = e
            self._agree(err, "self-check")

    def _agree(self, err, what):
        ok = 1 if err is None else 0
        if self.world > 1:
            be = str(dist.get_backend(self.group))
            t = torch.tensor([ok], dtype=torch.int32, device="cpu" if "gloo" in be else self.device)
            dist.all_reduce(t, op=dist.ReduceOp.MIN, group=self.group)
            ok = int(t.item())
        if not ok:
            self.close()
            raise RuntimeError("IpcComm %s failed on %s: %s" % (what, "this rank" if err else "a peer rank", err))

    def set_max_blocks(self, n: int, upto_bytes: int = -1):
        """Grid cap of the following launches of at most `upto_bytes` (-1: all; the same values on
        every rank)."""
        torch.ops.dtfe.ipc_set_max_blocks(self.handle, int(n), int(upto_bytes))

    def fits(self, t: torch.Tensor) -> bool:
        return t.numel() * t.element_size() + 64 <= self.cap and t.dtype in (torch.bfloat16, torch.float32)

    def all_reduce(self, t: torch.Tensor):
        """In-place sum over the group on the current stream (capturable)."""
        if not self.fits(t):
            if self.fallback is None:
                raise ValueError("IpcComm: %d B %s tensor exceeds the %d B staging buffer"
                                 % (t.numel() * t.element_size(), t.dtype, self.cap))
            self.fallback.all_reduce(t)
            return
        torch.ops.dtfe.ipc_all_reduce(t, self.handle)

    def status(self) -> int:
        """0 healthy, 1 a barrier timed out (synchronizes the device)."""
        return int(torch.ops.dtfe.ipc_status(self.handle))

    def check(self):
        """Sum rank-dependent data of a few shapes / alignments / dtypes and compare."""
        W = self.world
        for n, off, dt in ((1, 0, torch.float32), (4099, 1, torch.bfloat16), (65536 + 5, 3, torch.float32),
                           (1 << 20, 0, torch.bfloat16)):
            base = torch.empty(n + 8, device=self.device, dtype=dt)
            x = base[off:off + n]
            if not self.fits(x):
                continue
            idx = torch.arange(n, device=self.device, dtype=torch.float32)
            x.copy_(((idx % 13) + self.rank + 1).to(dt))
            self.all_reduce(x)
            exp = ((idx % 13) * W + W * (W + 1) / 2).to(dt)
            if self.status() != 0:
                raise RuntimeError("IpcComm self-check: a peer did not reach the barrier (timeout)")
            if not torch.equal(x, exp):
                bad = int((x != exp).sum().item())
                raise RuntimeError("IpcComm self-check: %d of %d elements wrong (n=%d, offset=%d, %s)"
                                   % (bad, n, n, off, dt))

    def close(self):
        if getattr(self, "handle", None) is not None:
            torch.ops.dtfe.ipc_destroy(self.handle)
            self.handle = None
