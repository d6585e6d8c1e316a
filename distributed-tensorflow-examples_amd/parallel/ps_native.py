"""Native single-node parameter-server data plane (csrc/bindings/ps_ops.cpp).

The reference moves every variable from the ps task to the worker and every gradient back
through TF's gRPC RecvTensor path on every ``sess.run`` (gan/distributed_gan.py:193,
encoder/distributed_encoder.py:165).  On one MI355X node this module replaces that with:

* ps side (``NativeShardService``): per worker a gradient mailbox and a parameter reply buffer
  in the ps GPU's HBM (one uncached hipIpc allocation), a shared request/reply page, and a C++
  progress thread that applies every arriving mailbox with the fused TF1 optimizer kernels;
  the apply writes the updated bf16 working copies (and fp32 variables) straight into that
  worker's reply buffer, and its last workgroup advances the step scalars and publishes the
  reply - no snapshot copy, no Python, no GIL, no host copies on the data path;
* worker side (``NativePSLink``): copy plans that push the gradient buckets straight from the
  worker's flat gradient buffer into its mailbox (fp32 -> bf16 in flight for bf16-compute
  models) and pull the reply buffer straight into the worker's bf16 working copies (+ fp32
  masters of the fp32 variables); the request / wait are two one-thread kernels, so a whole
  worker step - forward, backward with the bucket pushes overlapping it on a side stream,
  request, wait, pull - is one hipGraph replay.  ``launch(i)`` / ``wait()`` are the
  ``BucketAllReduce`` hooks the step programs already call during backward.

Consistency of an async exchange (what a pull returns), against the reference's async PS where
every ``ApplyAdam`` / ``ApplyRMSProp`` reads the shared ``beta*_power`` / slots at its own time
and a pull reads each variable's value at pull time (gan/distributed_gan.py:158-159,193):

* a worker's gradient buckets may be applied at different moments (bucket 0 during its backward,
  the rest at its request).  Every range apply of one push uses the step scalars as they are at
  that apply (``skip_advance``), and the push's last launch advances them once - so with several
  workers, another worker's advance can fall between the two buckets of one push and the two
  ranges see different Adam beta powers.  TF1 behaves the same way (each variable's ApplyAdam
  reads the shared beta powers independently, ``use_locking=False``); with one worker, or with
  the whole push applied at the request (the default for a ps on the worker's own GPU), every
  range of a push sees the same scalars;
* a range's reply values are written when that worker's own apply of it runs (fused replies) or
  copied right after it; if ANOTHER worker applied an overlapping range after that, the range
  is copied again at this worker's request (``refreshed_ranges`` in ``stats()``), so a pull
  returns the values current at reply time, as the reference's does.  --hogwild applies race by
  design and are not refreshed.

Everything is keyed by the cluster spec in the TCPStore (shm name, IPC handle, buffer
sizes), and each shard's layout is the same ``FlatParams`` offsets on both sides, so a worker
needs no gather / scatter index tensors.  Control messages (INIT, SAVE, SET_STATE, STATUS,
DONE) keep the gloo channel of ``parallel/ps.py``; they pause the service around any access
to the shard.  Multi-node clusters and CPU runs keep the gloo transport.
"""
from __future__ import annotations

import contextlib
import os
import socket

import torch

from .. import ops
from ..optim import FlatParams

SLOT_BYTES = 256  # ps_link.h PS_SLOT_WORDS * 8
MAX_BUCKETS = 4   # ps_link.h PS_MAX_BUCKETS
ALIGN = 256  # bytes: every segment of a mailbox / reply buffer starts 256-B aligned
COPY_CHUNK = 16384
MODE = {("f32", "f32"): 0, ("f32", "bf16"): 1, ("bf16", "bf16"): 2, ("bf16", "f32"): 3}


def _round(n, a=ALIGN):
    return (n + a - 1) // a * a


def push_dtype(specs) -> str:
    """Wire dtype of a shard's gradients: bf16 for models that compute in bf16 (their weights
    carry bf16 working copies - the CNN / ResNets), fp32 for the fp32 reference models."""
    return "bf16" if any(s.bf16 for s in specs) else "f32"


def reply_layout(specs):
    """[(var name, part, byte offset, elements, dtype)] of a reply buffer: the bf16 working
    copies a bf16-compute variable is read through (natural + transposed), the fp32 master
    of every other variable."""
    out, off = [], 0
    for s in specs:
        parts = []
        if s.bf16:
            parts.append(("w16", "bf16"))
        if s.transpose is not None:
            parts.append(("wt16", "bf16"))
        if not parts:
            parts.append(("master", "f32"))
        for part, dt in parts:
            out.append((s.name, part, off, s.numel, dt))
            off = _round(off + s.numel * (2 if dt == "bf16" else 4))
    return out, max(off, ALIGN)


def shard_sizes(specs):
    lay = FlatParams(specs, "cpu", init=False)
    esz = 2 if push_dtype(specs) == "bf16" else 4
    mailbox = _round(lay.total * esz, 4096)
    _, reply = reply_layout(specs)
    return lay, mailbox, _round(reply, 4096)


def eligible(server, device) -> bool:
    """Native transport: every task on this host, driving GPUs."""
    if torch.device(device).type != "cuda":
        return False
    host = socket.gethostname()
    idents = [server._dev_ident[r] for r in range(server.world)]
    return all(i.startswith(host + "/cuda") for i in idents)


def _key(server, k, what):
    return "dtfe/psn/%d/%s" % (k, what)


def _part_tensor(P, name, part):
    if part == "w16":
        return P.w16[name]
    if part == "wt16":
        return P.wt16[name]
    return P.view(name)


class NativeShardService:
    """ps task side: the shard's mailboxes / reply buffers, shared page and progress thread."""

    def __init__(self, server, shard, num_workers: int, sync: bool = False, replicas_to_aggregate=None,
                 hogwild: bool = False, timeout_s: float = 60.0, fused_replies: bool = True,
                 stream: str = "normal"):
        """``fused_replies``: async applies write each worker's reply buffer themselves (default);
        False keeps the snapshot copies (bitwise the same pulls - tests/test_cluster_gpu.py).
        ``stream``: the apply stream - "normal", "high" (highest queue priority) or "cu<N>" (a
        mask of N CUs), for a ps sharing its GPU with a worker (bench.py --ps_stream)."""
        ops.require()
        lib = torch.ops.dtfe
        self.lib = lib
        self.server = server
        self.shard = shard
        self.k = server.task_index
        self.nw = num_workers
        dev = shard.device
        specs = shard.P.specs
        self.lay, self.mb, self.rb = shard_sizes(specs)
        self.dtype = push_dtype(specs)
        host, port = server.cluster.store_address()
        self.shm_name = "/dtfe_ps_%d_%d_%d" % (port, self.k, os.getpid())
        self.shm = lib.ps_shm_create(self.shm_name, num_workers * SLOT_BYTES)
        self.buf = lib.ps_ipc_alloc(num_workers * (self.mb + self.rb), dev.index or 0)
        base = lib.ps_ipc_ptr(self.buf)
        R = replicas_to_aggregate or num_workers
        self.svc = lib.ps_service_create(self.shm, num_workers, dev.index or 0, sync, R, hogwild)
        lib.ps_service_set_fused(self.svc, bool(fused_replies))
        prio, cus = (1, 0) if stream == "high" else ((0, int(stream[2:])) if stream.startswith("cu") else (0, 0))
        lib.ps_service_set_stream(self.svc, prio, cus)
        g16 = self.dtype == "bf16"
        last = len(shard.opts) - 1
        for i, o in enumerate(shard.opts):
            c = o.cfg
            gs = shard.gs if (shard.gs is not None and i == last) else None
            lib.ps_service_add_group(self.svc, o.kind, shard.P.master, o.s1, o.s2, c.lr, c.beta1, c.beta2,
                                     c.resolved_eps(), c.momentum, c.rho, o.beta_pow, gs,
                                     shard.gs_increments if gs is not None else 0, o._blob, o.nseg, o.nwork, g16)
        if shard.gs is not None:
            lib.ps_service_set_gs(self.svc, shard.gs)
        # async: pushes arrive bucket by bucket (ranges of this shard's flat layout) and are applied
        # as they land, while the worker is still in backward; the request applies what is left
        lib.ps_service_set_total(self.svc, self.lay.total)
        self.acc = None
        if sync:
            self.acc = torch.zeros(self.lay.total, dtype=torch.float32, device=dev)
            lib.ps_service_set_acc(self.svc, self.acc)
        layout, _ = reply_layout(specs)
        self._plans = []
        for w in range(num_workers):
            rbase = base + w * (self.mb + self.rb) + self.mb
            segs = []
            for name, part, off, n, dt in layout:
                src = _part_tensor(shard.P, name, part)
                segs.append([src.data_ptr(), rbase + off, n, MODE[(dt, dt)]])
            st = torch.tensor(segs, dtype=torch.int64)
            blob = lib.ps_plan(st, COPY_CHUNK, shard.P.master)
            self._plans.append(blob)
            lib.ps_service_set_worker(self.svc, w, base + w * (self.mb + self.rb), blob, len(segs),
                                      lib.ps_plan_nwork(st, COPY_CHUNK))
            # each segment's shard-flat variable offset: a bucket's variables are snapshotted into
            # the reply buffer right after the bucket's apply (async), not all at the reply
            lib.ps_service_set_snap_offsets(self.svc, w, torch.tensor(
                [self.lay.offsets[name] for name, _, _, _, _ in layout], dtype=torch.int64))
        torch.cuda.synchronize(dev)
        st = server.store
        st.set(_key(server, self.k, "shm"), self.shm_name)
        st.set(_key(server, self.k, "ipc"), bytes(lib.ps_ipc_handle(self.buf).numpy().tobytes()).hex())
        st.set(_key(server, self.k, "sizes"), "%d,%d,%s" % (self.mb, self.rb, self.dtype))
        lib.ps_service_start(self.svc)
        self.started = True

    @contextlib.contextmanager
    def paused(self):
        """Hold the progress thread (its streams drained) while a control handler touches the shard."""
        self.lib.ps_service_pause(self.svc)
        try:
            yield
            torch.cuda.synchronize(self.shard.device)
        finally:
            self.lib.ps_service_resume(self.svc)

    def stats(self):
        r, a, s, v, b, f = [int(x) for x in self.lib.ps_service_stats(self.svc)]
        return {"requests": r, "applies": a, "stale": s, "version": v, "bucket_applies": b, "refreshed_ranges": f}

    def stop(self):
        if getattr(self, "started", False):
            self.lib.ps_service_stop(self.svc)
            self.started = False
            torch.cuda.synchronize(self.shard.device)
            self.lib.ps_ipc_close(self.buf)
            self.lib.ps_shm_close(self.shm)


class NativePSLink:
    """Worker side: push / pull plans into every shard's mailbox / reply buffer of this worker.

    Has the ``BucketAllReduce`` step-program interface (``launch(i)``, ``wait()``, ``ready``,
    ``flush``, ``grad16 = None``): buckets are contiguous ranges of the worker's flat gradient
    buffer; ``launch(i)`` enqueues bucket i's push on a side stream forked from the compute
    stream (so it overlaps the rest of backward), ``wait()`` joins it and issues the request /
    wait / pull on the compute stream.  All of it is capturable."""

    grad16 = None

    def __init__(self, server, full: FlatParams, placement: dict, shard_specs: dict, gs_ps_task: int, device,
                 buckets=None, timeout_s: float = 60.0, overlap=None):
        """``overlap``: announce pushed buckets so the ps applies them during backward - None: only
        to ps tasks on another GPU than this worker's (True / False: always / never)."""
        ops.require()
        lib = torch.ops.dtfe
        self.lib = lib
        self.full = full
        self.device = torch.device(device)
        self.w = server.task_index
        self.timeout_s = timeout_s
        self.shards = []
        overlap_arg = overlap
        st = server.store
        for k, specs in sorted(shard_specs.items()):
            if not specs:
                continue
            name = st.get(_key(server, k, "shm")).decode()
            handle = bytes.fromhex(st.get(_key(server, k, "ipc")).decode())
            mb, rb, dt = st.get(_key(server, k, "sizes")).decode().split(",")
            mb, rb = int(mb), int(rb)
            lay, mb2, rb2 = shard_sizes(specs)
            assert (mb, rb, dt) == (mb2, rb2, push_dtype(specs)), "ps / worker disagree on the shard layout"
            n_workers = len(server.cluster.worker)
            shm = lib.ps_shm_open(name, n_workers * SLOT_BYTES)
            buf = lib.ps_ipc_open(torch.frombuffer(bytearray(handle), dtype=torch.uint8), self.device.index or 0)
            base = lib.ps_ipc_ptr(buf) + self.w * (mb + rb)
            # a ps task on this worker's own GPU: its applies would only compete with this worker's
            # backward for the CUs (bucket 0's apply stretched from 18 to 55-100 us beside the conv
            # backward, profiles/r4_ps_1p1w_timeline.txt), so no bucket is announced to it - the
            # request applies the whole push at once, while this worker waits
            overlap = not server.colocated(server.cluster.rank_of("ps", k), server.rank) if overlap_arg is None \
                else bool(overlap_arg)
            self.shards.append(dict(k=k, specs=specs, lay=lay, shm=shm, buf=buf, mailbox=base, reply=base + mb, dt=dt,
                                    overlap=overlap))
        self.gs_slot = next((i for i, sh in enumerate(self.shards) if sh["k"] == gs_ps_task), -1)
        # pull plan: reply buffers -> local working copies / masters (one launch for all shards)
        segs = []
        for sh in self.shards:
            layout, _ = reply_layout(sh["specs"])
            for name, part, off, n, dt in layout:
                dst = _part_tensor(full, name, part)
                segs.append([sh["reply"] + off, dst.data_ptr(), n, MODE[(dt, dt)]])
        self._pull = self._plan(segs)
        self.buckets = list(buckets) if buckets is not None else [(0, full.total)]
        self._push = [self._push_plan(lo, hi) for lo, hi in self.buckets]
        # per bucket and shard: the shard-flat range the bucket's variables occupy (the shard keeps
        # the full layout's variable order, so it is contiguous); announced after the bucket's push
        # so the ps applies it while backward continues.  More buckets than the slot has room for:
        # no announcements, the ps applies the whole push at the request.
        self._bkt_ranges = [self._shard_ranges(lo, hi) for lo, hi in self.buckets] \
            if len(self.buckets) <= MAX_BUCKETS else None
        self.side = torch.cuda.Stream(device=self.device)
        self.ctr = torch.zeros(1, dtype=torch.int64, device=self.device)
        # one version per shard: shard k's last reply version is the staleness tag of the next
        # request to shard k (sync mode drops pushes computed from an older version)
        self.ver = torch.zeros(max(1, len(self.shards)), dtype=torch.int64, device=self.device)
        self.gs_dev = torch.zeros(1, dtype=torch.int32, device=self.device)
        self.err = torch.zeros(1, dtype=torch.int32, device=self.device)
        self.seq = 0          # host mirror of ctr (requests issued, eager or replayed)
        self._forked = False
        self._launched = set()
        self._exchanged = False
        self.global_step = 0
        self.version = 0

    def _plan(self, segs):
        if not segs:
            return None
        st = torch.tensor(segs, dtype=torch.int64)
        return (self.lib.ps_plan(st, COPY_CHUNK, self.full.master), len(segs), self.lib.ps_plan_nwork(st, COPY_CHUNK))

    def _push_plan(self, lo, hi):
        """Gradient segments of every variable whose flat range lies in [lo, hi)."""
        segs = []
        for sh in self.shards:
            esz, mode = (2, MODE[("f32", "bf16")]) if sh["dt"] == "bf16" else (4, MODE[("f32", "f32")])
            for s in sh["specs"]:
                o = self.full.offsets[s.name]
                if lo <= o < hi:
                    segs.append([self.full.grad[o:o + s.numel].data_ptr(), sh["mailbox"] + sh["lay"].offsets[s.name] * esz,
                                 s.numel, mode])
        return self._plan(segs)

    def _shard_ranges(self, lo, hi):
        out = []
        for sh in self.shards:
            offs = [(sh["lay"].offsets[s.name], s.numel) for s in sh["specs"] if lo <= self.full.offsets[s.name] < hi]
            out.append((min(o for o, _ in offs), max(o + n for o, n in offs)) if offs else None)
        return out

    def _run(self, plan):
        if plan is not None:
            self.lib.ps_copy(plan[0], plan[1], plan[2])

    # ---- BucketAllReduce interface (called by the step programs during backward)
    def launch(self, i: int, after=None):
        """Push bucket i (once per step) on the side stream, forked from the current stream
        (and after the events ``after``: gradients produced on another stream)."""
        if i in self._launched:
            return
        self._launched.add(i)
        self.side.wait_stream(torch.cuda.current_stream(self.device))
        for ev in after or ():
            self.side.wait_event(ev)
        with torch.cuda.stream(self.side):
            self._run(self._push[i])
            # the step's last bucket is not announced: the request that follows it makes the ps
            # apply it in the launch that also advances the step scalars and writes the reply
            if self._bkt_ranges is not None and len(self._launched) < len(self.buckets):
                for sh, r in zip(self.shards, self._bkt_ranges[i]):
                    if r is not None and sh["overlap"]:
                        self.lib.ps_bucket(sh["shm"], self.w, self.ctr, i, r[0], r[1])
        self._forked = True

    def ready(self, lo: int, after=None):
        """Backward progress hook: every bucket starting at or above flat offset ``lo`` is final."""
        for i, (blo, _hi) in enumerate(self.buckets):
            if blo >= lo:
                self.launch(i, after)

    def flush(self):
        for i in range(len(self.buckets)):
            self.launch(i)

    def wait_bucket(self, i: int):
        self.wait_launched()

    def wait_launched(self):
        if self._forked:
            torch.cuda.current_stream(self.device).wait_stream(self.side)
            self._forked = False

    def wait(self):
        """Join the pushes, then request / wait / pull on the compute stream (once per step)."""
        if self._exchanged:
            return
        self.flush()
        self.wait_launched()
        self._exchange(1)
        self._exchanged = True

    def end_step(self):
        """Finish this step's exchange (a no-op if the program already did it inside backward)
        and re-arm the link for the next step."""
        self.wait()
        self._launched.clear()
        self._exchanged = False

    def _exchange(self, kind: int):
        # ONE request number per exchange for every shard (the first request bumps the counter,
        # the rest reuse it), so ps_wait's target matches what each shard answers
        for i, sh in enumerate(self.shards):
            self.lib.ps_request(sh["shm"], self.w, self.ctr, self.ver, kind, i, 1 if i == 0 else 0)
        self.lib.ps_wait([sh["shm"] for sh in self.shards], self.w, self.gs_slot, self.ctr, self.gs_dev, self.ver,
                         self.err, self.timeout_s)
        self._run(self._pull)

    # ---- host side
    def note_request(self):
        """One request was issued on the device (an eager exchange or a graph replay)."""
        self.seq += 1

    def host_reply(self):
        """Spin (host) until the ps answered request ``seq`` of every shard; returns the global step."""
        gs = self.global_step
        for i, sh in enumerate(self.shards):
            r = self.lib.ps_shm_wait_reply(sh["shm"], self.w, self.seq, self.timeout_s)
            if i == self.gs_slot:
                gs = int(r[0])
            if i == 0:
                self.version = int(r[1])
        self.global_step = gs
        return gs

    def check(self):
        if int(self.err.item()) != 0:
            raise RuntimeError("native ps link: no reply from a parameter server within %.0f s" % self.timeout_s)

    def pull(self) -> int:
        """Eager pull-only exchange (initial / evaluation reads of the variables)."""
        self._exchange(2)
        self.note_request()
        gs = self.host_reply()
        torch.cuda.current_stream(self.device).synchronize()
        self.check()
        return gs

    def push_pull(self) -> int:
        """Eager push of every bucket + exchange (steps that are not graph-captured)."""
        self.end_step()
        self.note_request()
        return self.host_reply()

    def close(self):
        torch.cuda.synchronize(self.device)
        for sh in self.shards:
            self.lib.ps_ipc_close(sh["buf"])
            self.lib.ps_shm_close(sh["shm"])
        self.shards = []
