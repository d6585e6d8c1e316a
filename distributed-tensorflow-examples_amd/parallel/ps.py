"""Parameter-server service and client.

Between-graph replication as in the reference (GAN:119-121, GAN:170-206), with
the TF runtime's implicit machinery made explicit:

* every ps task owns the variables ``placement.round_robin`` assigns to it
  (a FlatParams shard) plus their optimizer slots, and applies updates with
  the fused TF1 optimizer kernels (``apply_gradients``);
* every (ps, worker) pair has a private 2-rank channel (process group);
  workers never talk to each other (``device_filters``, GAN:179);
* one service thread per worker channel: it receives a request header,
  then the payload, applies / accumulates, and replies with fresh parameters
  and the global step - the Send/Recv pair of a ``sess.run``;
* ``global_step`` lives on the ps that owns its creation ordinal and is
  advanced by that shard's apply (TF's AssignAdd colocated with it);
* async mode (reference): apply on arrival.  Updates of one shard are
  serialised by a lock (deterministic), or lock-free with ``hogwild=True``
  (TF's ``use_locking=False`` race);
* sync mode ([NS], TF SyncReplicasOptimizer semantics): gradients tagged with
  the shard version the worker computed them from are accumulated; stale ones
  are dropped; after ``replicas_to_aggregate`` fresh ones the mean is applied,
  the version advances and every waiting worker is released (its "token");
* done protocol (C07): a DONE message per worker; the ps prints
  ``ps %d received done %d`` and quits after ``num_workers`` of them.

Request header (int64[4]): (type, tag, n_payload, reserved).
Reply header   (int64[4]): (global_step or -1, initialized, version, reserved).
"""
from __future__ import annotations

import threading
import time

import torch
import torch.distributed as dist

from ..optim import FlatParams, Optimizer

PULL, PUSH, INIT, SAVE, DONE, STATUS, SET_STATE = 1, 2, 3, 4, 5, 6, 7


class Shard:
    """Variables + optimizer state hosted by one ps task."""

    def __init__(self, specs, opt_groups, device, gs_here: bool, gs_increments: int):
        self.P = FlatParams(specs, device, init=False)
        self.names = [s.name for s in specs]
        self.device = torch.device(device)
        self.gs = torch.zeros(1, dtype=torch.int32, device=self.device) if gs_here else None
        self.gs_increments = gs_increments
        self.opts = []
        for cfg, var_list, bp_names in opt_groups:
            mine = [v for v in var_list if v in self.names]
            if mine:
                # the last optimizer of the step advances global_step on the owning shard
                self.opts.append(Optimizer(cfg, self.P, var_list=mine, global_step=None, beta_power_names=bp_names))
        self.initialized = False
        self.version = 0
        self.lock = threading.Lock()

    # payload layout == FlatParams master layout of this shard
    @property
    def numel(self):
        return self.P.total

    def apply(self, grad: torch.Tensor, scale: float = 1.0):
        """Apply one gradient payload (this shard's flat layout).  The payload goes to the
        optimizer kernels directly - never staged in a shared buffer - so concurrent (hogwild)
        applies race only on the variables and slots, as TF's use_locking=False does, and every
        pushed gradient is applied exactly once."""
        for o in self.opts:
            o.step(grad=grad, gscale=scale, gs_inc=0)
        if self.gs is not None:
            self.gs += self.gs_increments
        self.version += 1

    def reset_optimizer_state(self):
        for o in self.opts:
            if o.s1 is not None:
                o.s1.fill_(1.0 if o.cfg.kind == "rmsprop" else 0.0)
            if o.s2 is not None:
                o.s2.zero_()
            if o.beta_pow is not None:
                o.beta_pow[0] = o.cfg.beta1
                o.beta_pow[1] = o.cfg.beta2
        if self.gs is not None:
            self.gs.zero_()
        self.version = 0

    def global_step(self) -> int:
        return int(self.gs.item()) if self.gs is not None else -1

    def slot_tensors(self):
        out = {}
        for o in self.opts:
            out.update(o.slot_tensors())
        return out

    def state_payload(self):
        """params + every slot buffer, flattened (SAVE reply / SET_STATE payload)."""
        bufs = [self.P.master]
        for o in self.opts:
            bufs += [b for b in (o.s1, o.s2) if b is not None]
            if o.beta_pow is not None:
                bufs.append(o.beta_pow)
        return torch.cat([b.reshape(-1).float() for b in bufs])

    def load_state_payload(self, flat: torch.Tensor):
        off = 0
        n = self.P.total
        self.P.master.copy_(flat[off:off + n])
        off += n
        for o in self.opts:
            for b in (o.s1, o.s2):
                if b is not None:
                    b.copy_(flat[off:off + b.numel()])
                    off += b.numel()
            if o.beta_pow is not None:
                o.beta_pow.copy_(flat[off:off + 2])
                off += 2
        self.P.refresh_copies()

    def state_numel(self):
        n = self.P.total
        for o in self.opts:
            n += sum(b.numel() for b in (o.s1, o.s2) if b is not None)
            n += 2 if o.beta_pow is not None else 0
        return n


class PSServer:
    """The ps role of ``main(_)`` (GAN:108-117) plus the TF runtime's variable service."""

    def __init__(self, server, shard: Shard, num_workers: int, sync: bool = False, replicas_to_aggregate=None,
                 hogwild: bool = False, comm_device="cpu", log=print, watchdog=None, faults=None):
        self.server = server
        self.shard = shard
        self.num_workers = num_workers
        self.sync = sync
        self.R = replicas_to_aggregate or len(server.cluster.worker)
        self.hogwild = hogwild
        self.comm_device = torch.device(comm_device)
        self.log = log
        self.done_count = 0
        self._done_cv = threading.Condition()
        self._acc = None
        self._acc_n = 0
        self._acc_cv = threading.Condition()
        self._threads = []
        self.errors = []
        self.watchdog = watchdog      # health.Watchdog over the workers (None: reference semantics)
        self.faults = faults          # utils.faults.FaultInjector of this ps task
        self.done_ranks = set()
        self.lost = set()
        self.native = None            # ps_native.NativeShardService when PUSH/PULL use the native plane

    def _guard(self):
        """Exclusive access to the shard for a control handler (the native service pauses)."""
        if self.native is None:
            return self.shard.lock
        nat, lock = self.native, self.shard.lock

        class _G:
            def __enter__(self_):
                lock.acquire()
                self_.cm = nat.paused()
                self_.cm.__enter__()

            def __exit__(self_, *exc):
                try:
                    self_.cm.__exit__(*exc)
                finally:
                    lock.release()
        return _G()

    # ---- per-worker service thread
    def _serve(self, worker_rank: int):
        g = self.server.pair(self.server.rank, worker_rank)
        sh = self.shard
        cdev = self.server.pair_comm_device(self.server.rank, worker_rank, self.comm_device)
        hdr = torch.zeros(4, dtype=torch.int64)
        pay = torch.zeros(sh.numel, dtype=torch.float32, device=cdev)
        try:
            while True:
                dist.recv(hdr, src=worker_rank, group=g)
                typ, tag = int(hdr[0]), int(hdr[1])
                if typ == DONE:
                    with self._done_cv:
                        i = self.done_count
                        self.done_count += 1
                        self.done_ranks.add(worker_rank)
                        self.log("ps %d received done %d" % (self.server.task_index, i))
                        self._done_cv.notify_all()
                    self._membership_changed()
                    return
                if typ == STATUS:
                    self._reply_hdr(worker_rank, g)
                    continue
                if typ == INIT:
                    # global_variables_initializer: params from the chief, slots / beta powers /
                    # global_step back to their initial values
                    dist.recv(pay, src=worker_rank, group=g)
                    with self._guard():
                        sh.P.master.copy_(pay.to(sh.device))
                        sh.P.refresh_copies()
                        sh.reset_optimizer_state()
                        sh.initialized = True
                    self._reply_hdr(worker_rank, g)
                    continue
                if typ == SET_STATE:
                    st = torch.zeros(sh.state_numel(), dtype=torch.float32, device=cdev)
                    gsv = torch.zeros(1, dtype=torch.int64)
                    dist.recv(st, src=worker_rank, group=g)
                    dist.recv(gsv, src=worker_rank, group=g)
                    with self._guard():
                        sh.load_state_payload(st.to(sh.device))
                        if sh.gs is not None:
                            sh.gs.fill_(int(gsv.item()))
                        sh.initialized = True
                    self._reply_hdr(worker_rank, g)
                    continue
                if typ == SAVE:
                    with self._guard():
                        st = sh.state_payload().to(cdev)
                    self._reply_hdr(worker_rank, g)
                    dist.send(st, dst=worker_rank, group=g)
                    continue
                if typ == PUSH:
                    dist.recv(pay, src=worker_rank, group=g)
                    if self.sync:
                        self._sync_push(pay, tag)
                    elif self.hogwild:
                        sh.apply(pay.to(sh.device))
                    else:
                        with sh.lock:
                            sh.apply(pay.to(sh.device))
                    if self.faults:
                        self.faults.step(sh.global_step())
                # PULL and PUSH both answer with fresh parameters
                with self._guard():
                    params = sh.P.master.to(cdev, copy=True)
                self._reply_hdr(worker_rank, g)
                dist.send(params, dst=worker_rank, group=g)
        except Exception as e:  # noqa: BLE001 - a worker vanished: keep serving the others
            self.errors.append((worker_rank, repr(e)))

    def _reply_hdr(self, worker_rank, g):
        sh = self.shard
        r = torch.tensor([sh.global_step(), int(sh.initialized), sh.version, 0], dtype=torch.int64)
        dist.send(r, dst=worker_rank, group=g)

    def _active_workers(self) -> int:
        return self.num_workers - self.done_count - len(self.lost)

    def _apply_accumulated(self):
        """Apply the mean of the accumulated gradients, release the waiters (caller holds _acc_cv)."""
        sh = self.shard
        with sh.lock:
            sh.apply(self._acc.to(sh.device), scale=1.0 / self._acc_n)
        self._acc.zero_()
        self._acc_n = 0
        self._acc_cv.notify_all()

    def _membership_changed(self):
        """A worker finished or was lost: in sync mode a round that can no longer reach
        replicas_to_aggregate fresh gradients is applied with the ones it has (else the workers
        waiting on it would block forever), and the native service's target shrinks."""
        if not self.sync:
            return
        with self._acc_cv:
            if self._acc_n > 0 and self._acc_n >= min(self.R, self._active_workers()):
                self._apply_accumulated()
            self._acc_cv.notify_all()
        if self.native is not None:
            with self.native.paused():
                torch.ops.dtfe.ps_service_set_replicas(self.native.svc, max(1, min(self.R, self._active_workers())))

    def _sync_push(self, pay, tag):
        sh = self.shard
        with self._acc_cv:
            if tag < sh.version:  # stale gradient: dropped (ConditionalAccumulator semantics)
                return
            if self._acc is None:
                self._acc = torch.zeros_like(pay)
            self._acc += pay
            self._acc_n += 1
            if self._acc_n >= min(self.R, max(1, self._active_workers())):
                self._apply_accumulated()
            else:
                v = sh.version
                while sh.version == v:
                    self._acc_cv.wait(timeout=1.0)
                    if sh.version == v and self._acc_n > 0 and self._acc_n >= min(self.R, max(1, self._active_workers())):
                        self._apply_accumulated()

    def serve_forever(self):
        for w in self.server.cluster.worker_ranks()[: len(self.server.cluster.worker)]:
            t = threading.Thread(target=self._serve, args=(w,), daemon=True, name="ps-serve-%d" % w)
            t.start()
            self._threads.append(t)
        cl = self.server.cluster
        with self._done_cv:
            while self.done_count + len(self.lost) < self.num_workers:
                self._done_cv.wait(timeout=1.0)
                if self.watchdog is None:
                    continue
                for _job, task, age in self.watchdog.poll():
                    if cl.rank_of("worker", task) in self.done_ranks or task in self.lost:
                        continue  # finished normally, then exited
                    self.lost.add(task)
                    self.log("ps %d: worker %d lost (no heartbeat for %.0fs)" % (self.server.task_index, task, age))
                    self._done_cv.release()
                    try:
                        self._membership_changed()
                    finally:
                        self._done_cv.acquire()
        self.log("ps %d: quitting" % self.server.task_index)


class PSClient:
    """Worker-side view of all ps shards (the variable reads / Apply sends of ``sess.run``)."""

    def __init__(self, server, full: FlatParams, placement: dict, shard_specs: dict, gs_ps: int,
                 opt_groups=(), comm_device="cpu"):
        self.server = server
        self._state_numel = {k: shard_state_numel(specs, opt_groups) for k, specs in shard_specs.items() if specs}
        self.full = full
        self.placement = placement
        self.comm_device = torch.device(comm_device)
        self.gs_ps = gs_ps
        self.lock = threading.Lock()  # one outstanding request per channel (chief's saver thread shares it)
        self.shards = {}
        for ps_task, specs in shard_specs.items():
            if not specs:
                continue
            layout = FlatParams(specs, "cpu", init=False)
            idx_src, idx_dst = [], []
            for s in specs:
                o_full = full.offsets[s.name]
                o_sh = layout.offsets[s.name]
                idx_src.append(torch.arange(o_full, o_full + s.numel))
                idx_dst.append(torch.arange(o_sh, o_sh + s.numel))
            ps_rank = server.cluster.rank_of("ps", ps_task)
            dev = server.pair_comm_device(ps_rank, server.rank, self.comm_device)
            self.shards[ps_task] = dict(
                rank=ps_rank, numel=layout.total, dev=dev,
                src=torch.cat(idx_src).to(full.device), dst=torch.cat(idx_dst).to(dev),
                buf=torch.zeros(layout.total, dtype=torch.float32, device=dev), layout=layout)
        self.versions = {k: 0 for k in self.shards}
        self.global_step = 0
        self.initialized = False

    def _g(self, ps_rank):
        return self.server.pair(ps_rank, self.server.rank)

    def _send_hdr(self, ps_rank, typ, tag=0, n=0):
        dist.send(torch.tensor([typ, tag, n, 0], dtype=torch.int64), dst=ps_rank, group=self._g(ps_rank))

    def _recv_hdr(self, ps_rank):
        h = torch.zeros(4, dtype=torch.int64)
        dist.recv(h, src=ps_rank, group=self._g(ps_rank))
        return [int(x) for x in h]

    def _gather(self, src_flat, sh):
        sh["buf"].zero_()
        sh["buf"][sh["dst"]] = src_flat[sh["src"]].to(sh["dev"])
        return sh["buf"]

    def _scatter_params(self, sh):
        self.full.master[sh["src"]] = sh["buf"][sh["dst"]].to(self.full.device)

    def _exchange(self, typ, grads=None):
        with self.lock:
            for k, sh in self.shards.items():
                self._send_hdr(sh["rank"], typ, tag=self.versions[k])
                if typ == PUSH:
                    dist.send(self._gather(grads, sh), dst=sh["rank"], group=self._g(sh["rank"]))
            for k, sh in self.shards.items():
                gs, init, ver, _ = self._recv_hdr(sh["rank"])
                dist.recv(sh["buf"], src=sh["rank"], group=self._g(sh["rank"]))
                self._scatter_params(sh)
                self.versions[k] = ver
                if sh["rank"] == self.gs_ps:
                    self.global_step = gs
                    self.initialized = bool(init)
        self.full.refresh_copies()
        return self.global_step

    def pull(self) -> int:
        return self._exchange(PULL)

    def push_pull(self, grads: torch.Tensor) -> int:
        return self._exchange(PUSH, grads)

    def status(self):
        """(initialized on every shard, global_step)"""
        with self.lock:
            ok = True
            gs = -1
            for sh in self.shards.values():
                self._send_hdr(sh["rank"], STATUS)
                g, init, _v, _ = self._recv_hdr(sh["rank"])
                ok = ok and bool(init)
                if sh["rank"] == self.gs_ps:
                    gs = g
            return ok, gs

    def init_variables(self):
        """Chief: push the locally initialised values to every shard (Supervisor init_op)."""
        with self.lock:
            for sh in self.shards.values():
                self._send_hdr(sh["rank"], INIT)
                dist.send(self._gather(self.full.master, sh), dst=sh["rank"], group=self._g(sh["rank"]))
            for sh in self.shards.values():
                self._recv_hdr(sh["rank"])

    def fetch_state(self):
        """Chief's saver: every shard's params + slots (per ps task) and the global step."""
        out = {}
        gs = -1
        with self.lock:
            for k, sh in self.shards.items():
                self._send_hdr(sh["rank"], SAVE)
            for k, sh in self.shards.items():
                g, _init, _v, _ = self._recv_hdr(sh["rank"])
                if sh["rank"] == self.gs_ps:
                    gs = g
                n = int(self._state_numel[k])
                st = torch.zeros(n, dtype=torch.float32, device=sh["dev"])
                dist.recv(st, src=sh["rank"], group=self._g(sh["rank"]))
                out[k] = st.cpu()
        return out, gs

    def set_state(self, states: dict, gs: int):
        """Chief restore: push params + slots + global_step to every shard."""
        with self.lock:
            for k, sh in self.shards.items():
                self._send_hdr(sh["rank"], SET_STATE)
                dist.send(states[k].to(sh["dev"]), dst=sh["rank"], group=self._g(sh["rank"]))
                dist.send(torch.tensor([gs], dtype=torch.int64), dst=sh["rank"], group=self._g(sh["rank"]))
            for sh in self.shards.values():
                self._recv_hdr(sh["rank"])

    def done(self):
        with self.lock:
            for sh in self.shards.values():
                self._send_hdr(sh["rank"], DONE)


def shard_state_numel(specs, opt_groups) -> int:
    """Size of a shard's SAVE payload: params + full-size slot buffers + beta powers (see Shard)."""
    total = sum((s.numel + FlatParams.ALIGN - 1) // FlatParams.ALIGN * FlatParams.ALIGN for s in specs)
    names = {s.name for s in specs}
    n = total
    for cfg, var_list, _bp in opt_groups:
        if not any(v in names for v in var_list):
            continue
        n += len(Optimizer.SLOT_NAMES[cfg.kind]) * total
        n += 2 if cfg.kind == "adam" else 0
    return n


def wait_for_init(client: PSClient, poll_s: float = 0.5, timeout_s: float = 3600.0, log=None):
    """Non-chief ``SessionManager.wait_for_session``: poll until the chief initialised every shard."""
    t0 = time.time()
    while True:
        ok, gs = client.status()
        if ok:
            return gs
        if time.time() - t0 > timeout_s:
            raise TimeoutError("variables not initialised by the chief within %.0fs" % timeout_s)
        if log:
            log("Waiting for model to be ready.")
        time.sleep(poll_s)
