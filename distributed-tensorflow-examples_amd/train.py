"""The shared ``main(_)`` of every example script.

``run(model_name, argv)`` reproduces the reference scripts' behaviour once,
for every model (the reference copy-pastes it three times, GAN/ENC/LSTM):

* ``--job_name=ps``: host this task's variable shard, serve the workers, count
  done signals (``ps %d received done %d`` / ``ps %d: quitting``);
* ``--job_name=worker``: build the step program, join the Supervisor (chief =
  task 0), pull -> compute gradients -> push/pull per step printing
  ``Global step %d Local step %d  AvgTime: %3.2fms``, print ``Total Time``,
  (LSTM) ``Test-Accuracy``, signal done to every ps, stop.

plus the north-star modes: ``--sync`` (sync SGD with a chief over the ps) and
``--mode=allreduce`` (ring all-reduce data parallelism, no ps).
"""
from __future__ import annotations

import contextlib
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

from . import ckpt
from .data import cifar, imagenet_synth
from .data.mnist import DeviceBatcher, read_data_sets as read_mnist
from .models.autoencoder import AutoencoderModel
from .models.base import ScaledScalar
from .models.gan import LR as GAN_LR, GanModel
from .models.lstm import LR as LSTM_LR, LstmModel
from .models.mnist_cnn import MnistCnnModel
from .models.resnet import ResNetModel
from .models.softmax_reg import SoftmaxRegressionModel
from .models.autoencoder import LR as ENC_LR
from .optim import Optimizer
from .parallel.allreduce import BucketAllReduce
from .parallel.comm import make_comm
from .parallel.cluster import ClusterSpec, Server
from .parallel.health import CommWatchdog, Heartbeat, Watchdog
from .utils.faults import FaultInjector
from .utils.timers import PhaseTimer
from .parallel.partition import PartitionedModel
from .parallel.placement import round_robin
from .parallel import ps_native
from .parallel.ps import PSClient, PSServer, Shard, wait_for_init
from .parallel.supervisor import Supervisor
from .utils import flags as flagmod
from .utils.graphs import StepGraph

MODELS = {
    "gan": (GanModel, GAN_LR),
    "encoder": (AutoencoderModel, ENC_LR),
    "lstm": (LstmModel, LSTM_LR),
    "softmax": (SoftmaxRegressionModel, 0.01),
    "cnn": (MnistCnnModel, 0.001),
    "resnet20": (lambda lr=0.1: ResNetModel(lr, "resnet20"), 0.1),
    "resnet50": (lambda lr=0.1: ResNetModel(lr, "resnet50"), 0.1),
}


def read_data_sets(model, data_dir, one_hot=True, seed=0, log=print):
    """The model's dataset: MNIST (reference models + CNN), CIFAR-10 (ResNet-20) or a
    synthetic ImageNet-shape set (ResNet-50)."""
    name = getattr(model, "name", "")
    if name == "resnet20":
        return cifar.read_data_sets(data_dir, one_hot=one_hot, seed=seed, log=log)
    if name == "resnet50":
        return imagenet_synth.read_data_sets(one_hot=one_hot, seed=seed, log=log)
    return read_mnist(data_dir, one_hot=one_hot, seed=seed, log=log)


def _print(*args):
    print(*args, flush=True)


def resolve_device(flag: str, local_rank: int = 0):
    if flag == "cpu" or (flag == "auto" and not torch.cuda.is_available()):
        return torch.device("cpu")
    if not torch.cuda.is_available():
        raise RuntimeError("--device=cuda but no GPU is visible")
    n = torch.cuda.device_count()
    return torch.device("cuda", local_rank % max(n, 1))


def resolve_backend(flag: str, device) -> str:
    if flag != "auto":
        return flag
    return "nccl" if device.type == "cuda" else "gloo"


# ------------------------------------------------------------------ logging
def step_line(step, local_step, ms, py2=False):
    parts = ("Global step %d" % step, "Local step %d" % local_step, " AvgTime: %3.2fms" % ms)
    return repr(parts) if py2 else " ".join(parts)


def scalar_metrics(metrics) -> dict:
    """Float scalars of a step's metrics (``loss``; GAN ``gen_loss`` / ``disc_loss``) as Python
    floats - the loss values written to the events file and the --metrics_jsonl stream."""
    out = {}
    for k, v in (metrics or {}).items():
        if isinstance(v, ScaledScalar) or (torch.is_tensor(v) and v.numel() == 1 and v.is_floating_point()):
            out[k] = float(v.item())
    return out


def model_step_hook(model, step, metrics, log):
    if model.name == "gan" and (step % 1000 == 0 or step == 1):
        log("Step %i: Generator Loss: %f, Discriminator Loss: %f"
            % (step, float(metrics["gen_loss"].item()), float(metrics["disc_loss"].item())))


class MetricsLog:
    def __init__(self, path):
        self.f = open(path, "a") if path else None

    def write(self, **kw):
        if self.f:
            self.f.write(json.dumps(kw) + "\n")
            self.f.flush()


# ---------------------------------------------------------------- batching
class Feeder:
    """next batch for a program: host next_batch on CPU, HBM gather on GPU."""

    def __init__(self, data, program, device):
        self.B = program.batch_size
        self.dev = None
        if device.type == "cuda":
            self.dev = DeviceBatcher(data.train, device, self.B, one_hot=True)
        self.data = data

    def next(self):
        if self.dev is not None:
            return self.dev.next_batch()
        x, y = self.data.train.next_batch(self.B)
        return torch.from_numpy(x), torch.from_numpy(y)


# ---------------------------------------------------------- checkpoint glue
def var_list(model):
    shapes = model.tf_shapes()
    out = []
    for n in model.var_order:
        if n == model.gs_name:
            out.append((n, ckpt.DT_INT32, []))
        else:
            out.append((n, ckpt.DT_FLOAT, list(shapes[n])))
    return out


def tensors_from_flat(model, P, optimizers, gs: int):
    """Checkpoint dict (TF names and layouts) from a FlatParams + its optimizers."""
    out = {}
    for s in model.specs:
        if s.name in P.offsets:  # a ps shard holds a subset
            out[s.name] = model.to_tf(s.name, P.view(s.name).detach().cpu())
    for o in optimizers:
        for k, t in o.slot_tensors().items():
            base = k.rsplit("/", 1)[0]  # "<var>/Adam" -> "<var>"; beta powers have no slash
            if "/" in k and base in P.offsets:
                t = model.to_tf(base, t)
            out[k] = t
    out[model.gs_name] = torch.tensor(int(gs), dtype=torch.int32)
    return out


def load_flat_from_tensors(model, P, optimizers, tensors):
    for s in model.specs:
        if s.name in tensors and s.name in P.offsets:
            P.view(s.name).copy_(model.from_tf(s.name, tensors[s.name]).reshape(s.shape).to(P.device))
    conv = {}
    for k, t in tensors.items():
        if "/" in k:
            base = k.rsplit("/", 1)[0]
            if base in P.offsets:
                t = model.from_tf(base, t)
        conv[k] = t
    for o in optimizers:
        o.load_slot_tensors(conv)
    P.refresh_copies()
    return int(tensors.get(model.gs_name, torch.tensor(0)).item())


# --------------------------------------------------------------------- ps
def _shard_layout(model, num_ps):
    placement = round_robin(model.var_order, num_ps)
    shard_specs = {k: [s for s in model.specs if placement[s.name] == k] for k in range(num_ps)}
    return placement, shard_specs


def ps_view(flags, model):
    """The model as the ps tasks see it: with --ps_partition_mb, large variables split into
    partitions that are placed (and checkpointed) like TF's PartitionedVariable parts."""
    mb = getattr(flags, "ps_partition_mb", 0.0) or 0.0
    return PartitionedModel(model, int(mb * (1 << 20))) if mb > 0 else model


def run_ps(flags, model, server, device, log):
    model = ps_view(flags, model)
    placement, shard_specs = _shard_layout(model, len(server.cluster.ps))
    k = server.task_index
    gs_here = placement[model.gs_name] == k
    shard = Shard(shard_specs[k], model.opt_groups, device, gs_here, model.gs_increments)
    comm = "cpu" if server.backend == "gloo" else device
    hb = Heartbeat(server.store, "ps", k, flags.heartbeat_secs)
    wd = Watchdog(server.store, [("worker", i) for i in range(len(server.cluster.worker))],
                  flags.heartbeat_timeout) if flags.heartbeat_secs > 0 else None
    ps = PSServer(server, shard, num_workers=flags.workers, sync=flags.sync,
                  replicas_to_aggregate=flags.replicas_to_aggregate, hogwild=flags.hogwild, comm_device=comm,
                  log=log, watchdog=wd, faults=FaultInjector("ps", k, log=log))
    if _native_ps(flags, server, device):
        ps.native = ps_native.NativeShardService(server, shard, len(server.cluster.worker), sync=flags.sync,
                                                 replicas_to_aggregate=flags.replicas_to_aggregate,
                                                 hogwild=flags.hogwild)
    ps.serve_forever()
    if ps.native is not None:
        st = ps.native.stats()
        log("ps %d: native data plane: %d requests, %d applies (%d bucket applies during backward), %d stale"
            % (k, st["requests"], st["applies"], st["bucket_applies"], st["stale"]))
        ps.native.stop()
    hb.stop()
    if ps.lost:
        # service threads of lost workers are blocked in recv: leave without the collective teardown
        sys.stdout.flush()
        os._exit(0)
    # The ps hosts the TCPStore and owns nothing the job still needs once every worker has
    # said done (checkpoints are the chief's).  Tear the process groups down, then leave
    # without interpreter finalisation: static destructors of the communicator / store
    # threads racing the workers' own teardown end in std::terminate on a ROCm box.
    server.shutdown()
    sys.stdout.flush()
    sys.stderr.flush()
    os._exit(0)


def _native_ps(flags, server, device) -> bool:
    """Whether the ps roles move PUSH / PULL over the native single-node data plane."""
    if flags.ps_transport == "pg":
        return False
    ok = ps_native.eligible(server, device)
    if flags.ps_transport == "native" and not ok:
        raise SystemExit("--ps_transport=native needs every task on this host, on GPUs")
    return ok


def ps_state(client, model, shard_specs, placement):
    """Gather every shard's params + slots from the ps tasks into one TF-named dict (partitioned
    variables: one ``ckpt.Sliced`` per variable / slot)."""
    states, gs = client.fetch_state()
    out = {}
    for k, flat in states.items():
        mirror = Shard(shard_specs[k], model.opt_groups, "cpu", False, model.gs_increments)
        mirror.load_state_payload(flat)
        out.update(tensors_from_flat(model, mirror.P, mirror.opts, gs))
    out[model.gs_name] = torch.tensor(int(gs), dtype=torch.int32)
    if isinstance(model, PartitionedModel):
        out = model.merge_tf(out)
    return out, gs


def ps_restore(client, model, shard_specs, tensors):
    states = {}
    gs = int(tensors.get(model.gs_name, torch.tensor(0)).item())
    if isinstance(model, PartitionedModel):
        tensors = model.split_tf(tensors)
    for k, specs in shard_specs.items():
        if not specs:
            continue
        mirror = Shard(specs, model.opt_groups, "cpu", False, model.gs_increments)
        load_flat_from_tensors(model, mirror.P, mirror.opts, tensors)
        states[k] = mirror.state_payload()
    client.set_state(states, gs)


def run_worker_ps(flags, model, server, device, log):
    cl = server.cluster
    full_model, model = model, ps_view(flags, model)
    placement, shard_specs = _shard_layout(model, len(cl.ps))
    gs_rank = cl.rank_of("ps", placement[model.gs_name])
    prog = full_model.program(device, flags.batch_size, seed=flags.seed)
    if isinstance(model, PartitionedModel):
        model.add_aliases(prog.P)  # the parts as views of the worker's full variables
    comm = "cpu" if server.backend == "gloo" else device
    client = PSClient(server, prog.P, placement, shard_specs, gs_rank, model.opt_groups, comm_device=comm)
    is_chief = server.task_index == 0
    sv = Supervisor(
        is_chief, flags.model_dir,
        state_fn=lambda: ps_state(client, model, shard_specs, placement),
        restore_fn=lambda t: ps_restore(client, model, shard_specs, t),
        init_fn=client.init_variables,
        wait_fn=lambda: wait_for_init(client),
        var_list_fn=lambda: var_list(model),
        gs_fn=lambda: client.status()[1],
        save_model_secs=flags.save_model_secs, save_summaries_secs=flags.save_summaries_secs,
        max_to_keep=flags.max_to_keep, log=log)
    data = read_data_sets(model, "" if flags.synthetic else flags.data_dir, one_hot=True,
                          seed=flags.seed * 1000 + server.task_index + 1, log=log)
    feeder = Feeder(data, prog, device)
    metrics_log = MetricsLog(flags.metrics_jsonl)
    hb = Heartbeat(server.store, "worker", server.task_index, flags.heartbeat_secs)
    faults = FaultInjector("worker", server.task_index, log=log)
    begin_time = time.time()
    sv.prepare()
    if flags.reinit_on_join:
        # GAN:181 / ENC:160: every worker re-runs init, clobbering restore + progress
        prog.P.initialize(flags.seed)
        client.init_variables()
    link = None
    if _native_ps(flags, server, device):
        # gradient buckets in backward-completion order (flat order = the order backward produces them)
        link = ps_native.NativePSLink(server, prog.P, placement, shard_specs, placement[model.gs_name], device,
                                      buckets=_ps_buckets(prog, flags.bucket_mb))
        core = getattr(prog, "core", None)
        if core is not None and hasattr(core, "allreduce"):
            core.allreduce = link       # the CNN program pushes its buckets from inside backward
        elif hasattr(prog, "grad_ready"):
            prog.grad_ready = link.ready
    state = {}

    def native_step():
        state["m"] = prog.compute_grads()
        link.end_step()    # push what backward has not pushed yet, request / wait / pull

    runner = StepGraph(native_step, warmup=2, capture_error_mode="thread_local",
                       enabled=link is not None and flags.hip_graph) if link is not None else None
    if link is not None:
        link.pull()
    else:
        client.pull()
    step = 0
    local_step = 0
    try:
        while not sv.should_stop() and step < flags.num_steps:
            t0 = time.time()
            prog.load_batch(feeder.next())
            if link is not None:
                runner()
                link.note_request()
                step = link.host_reply()
                metrics = state.get("m")
                if local_step % flags.log_every == 0:
                    link.check()
                    prog.check_health()
            else:
                metrics = prog.compute_grads()
                step = client.push_pull(prog.P.grad)
            if flags.check_pull:
                log("pull checksum gs=%d: %.9e" % (step, float(prog.P.master.double().sum().item())))
            faults.step(step)
            elapsed = time.time() - t0
            ips = prog.batch_size / max(elapsed, 1e-9)
            sc = scalar_metrics(metrics)
            if local_step % flags.log_every == 0:
                log(step_line(step, local_step, elapsed * 1000, flags.py2_print))
                sv.summary(step, dict(sc, **{"images/sec": ips}))
            model_step_hook(model, step, metrics, log)
            metrics_log.write(step=local_step, gs=step, ms=elapsed * 1000, images_per_sec=ips, **sc)
            local_step += 1
        log("Total Time: %3.2fs" % float(time.time() - begin_time))
        if model.name in ("lstm", "cnn"):
            link.pull() if link is not None else client.pull()
            test_len = 128
            acc = prog.evaluate(torch.from_numpy(data.test.images[:test_len]).to(device),
                                torch.from_numpy(data.test.labels[:test_len]).to(device))
            log("Test-Accuracy: %2.4f" % acc)
        # the chief's checkpoint / step-counter threads talk to the ps: join them before the done
        # message (the last done makes the ps quit, and a save started after it fails on a closed
        # connection)
        sv.stop()
        client.done()
    finally:
        hb.stop()
        sv.stop()
        if link is not None:
            link.close()


# --------------------------------------------------------------- allreduce
def run_allreduce(flags, model, device, log, world=1, rank=0, group=None, store=None):
    prog = model.program(device, flags.batch_size, seed=flags.seed)
    gstep = torch.zeros(1, dtype=torch.int32, device=device)
    opts = []
    for i, (cfg, var_list_, bp) in enumerate(model.opt_groups):
        cfg.lr = flags.learning_rate if flags.learning_rate is not None else cfg.lr
        opts.append(Optimizer(cfg, prog.P, var_list=var_list_, global_step=gstep, beta_power_names=bp))
    is_chief = rank == 0
    sv = Supervisor(
        is_chief, flags.model_dir,
        state_fn=lambda: (tensors_from_flat(model, prog.P, opts, int(gstep.item())), int(gstep.item())),
        restore_fn=lambda t: gstep.fill_(load_flat_from_tensors(model, prog.P, opts, t)),
        init_fn=lambda: None, wait_fn=lambda: None, var_list_fn=lambda: var_list(model),
        gs_fn=lambda: int(gstep.item()),
        save_model_secs=flags.save_model_secs, save_summaries_secs=flags.save_summaries_secs,
        max_to_keep=flags.max_to_keep, log=log)
    sv.prepare()
    ar = None
    # programs with their own data-parallel schedule (the MNIST CNN: the one bench.py times) run it
    # here too, unless --bucket_mb asks for generic flat-buffer buckets
    native = (hasattr(prog, "attach_data_parallel") and len(opts) == 1
              and (world == 1 or flags.bucket_mb is None))
    if world > 1:
        # chief's (possibly restored) state is the starting point of every replica
        dist.broadcast(prog.P.master, src=0, group=group)
        dist.broadcast(gstep, src=0, group=group)
        for o in opts:
            for b in (o.s1, o.s2, o.beta_pow):
                if b is not None:
                    dist.broadcast(b, src=0, group=group)
        prog.P.refresh_copies()
        # on GPUs the buckets go through dtfe's own RCCL communicator (capturable: the whole step,
        # all-reduce included, replays as one hipGraph); gloo / CPU keeps ProcessGroup collectives
        bks = prog.core.buckets if native else _buckets(prog.P, flags.bucket_mb)
        comm = None
        # (gloo + --comm=ipc: several ranks sharing one GPU rehearse the in-graph IPC path)
        if device.type == "cuda" and flags.comm != "pg" and (dist.get_backend(group) != "gloo" or flags.comm == "ipc"):
            cdt = torch.bfloat16 if flags.comm_dtype == "bf16" else torch.float32
            comm = make_comm(device, group, [(hi - lo) * (2 if cdt == torch.bfloat16 else 4) for lo, hi in bks], cdt,
                             mode=flags.comm, log=log if is_chief else None,
                             timeout_s=flags.heartbeat_timeout if flags.heartbeat_secs > 0 else 30.0)
        ar = BucketAllReduce(prog.P.grad, bks, group=group, comm=comm,
                             comm_dtype=torch.bfloat16 if flags.comm_dtype == "bf16" else torch.float32)
        if not native and hasattr(prog, "grad_ready"):  # programs reporting backward progress overlap the all-reduce
            prog.grad_ready = ar.ready
    if native:
        prog.attach_data_parallel(ar, opts[0])
    data = read_data_sets(model, "" if flags.synthetic else flags.data_dir, one_hot=True, seed=flags.seed * 1000 + rank + 1,
                          log=log if is_chief else (lambda *_: None))
    feeder = Feeder(data, prog, device)
    metrics_log = MetricsLog(flags.metrics_jsonl)

    state = {}
    trace = flags.trace_json if world == 1 or not flags.trace_json else \
        flags.trace_json.replace(".json", "") + ".rank%d.json" % rank
    timer = PhaseTimer(device, trace_path=trace or None, rank=rank) \
        if (flags.phase_timers or flags.trace_json) else None
    phase = timer.phase if timer else (lambda _n: contextlib.nullcontext())
    faults = FaultInjector("worker", rank, log=log)
    # failure detection, on by default in this mode (utils/flags.py resolve_mode): every
    # rank beats into the TCPStore and a watchdog thread aborts the collectives and ends this rank when
    # a peer goes silent (or never beats) / the store vanishes / RCCL reports an error - the step graph
    # itself would wait on a dead peer forever
    hb = wd = None
    if world > 1 and store is not None and flags.heartbeat_secs > 0:
        hb = Heartbeat(store, "worker", rank, flags.heartbeat_secs)
        wd = CommWatchdog(store, "worker", rank, world, comm=ar.comm if ar is not None else None,
                          interval=min(1.0, flags.heartbeat_secs), timeout=flags.heartbeat_timeout, log=log)

    def train_step():
        if native:  # forward, backward, overlapped all-reduce and Adam in the program's own order
            with phase("step"):
                state["m"] = prog.train_step(grad16=ar.grad16 if ar is not None else None, gscale=1.0 / world)
            return
        with phase("fwd+bwd"):
            state["m"] = prog.compute_grads()
        g16 = None
        if ar is not None:
            with phase("comm"):
                ar.flush()
                ar.wait()
            g16 = ar.grad16
        with phase("apply"):
            # every minimize op of the step in one (grouped) launch; gs advances once per step by gs_increments
            Optimizer.step_all(opts, [model.gs_increments if i == len(opts) - 1 else 0 for i in range(len(opts))],
                               grad16=g16, gscale=1.0 / world)

    runner = StepGraph(train_step, warmup=2, capture_error_mode="thread_local",
                       enabled=(device.type == "cuda" and (world == 1 or ar.comm is not None) and flags.hip_graph
                                and timer is None))
    begin_time = time.time()
    step = int(gstep.item())
    local_step = 0
    try:
        while not sv.should_stop() and step < flags.num_steps:
            t0 = time.time()
            prog.load_batch(feeder.next())
            runner()
            step = int(gstep.item())
            faults.step(step)
            elapsed = time.time() - t0
            ips = prog.batch_size * world / max(elapsed, 1e-9)
            sc = scalar_metrics(state.get("m"))
            if local_step == 0 and native and ar is not None and is_chief:
                log("schedule: " + " < ".join(prog.core.schedule))
            if local_step % flags.log_every == 0:
                log(step_line(step, local_step, elapsed * 1000, flags.py2_print))
                if timer is not None:
                    log(PhaseTimer.format(timer.summary()))
                sv.summary(step, dict(sc, **{"images/sec": ips}))
                if ar is not None and ar.comm is not None:
                    ar.comm.check_health()  # IPC barrier timeouts fail the job on every rank
                prog.check_health()
            if "m" in state:
                model_step_hook(model, step, state["m"], log)
            metrics_log.write(step=local_step, gs=step, ms=elapsed * 1000, images_per_sec=ips, **sc)
            local_step += 1
        if wd is not None:  # training is over: peers may now leave at their own pace
            wd.stop()
            _leave_watchdog(store, rank, world, flags.heartbeat_timeout)
        if ar is not None and ar.comm is not None:
            ar.comm.check_health()
        prog.check_health()
        log("Total Time: %3.2fs" % float(time.time() - begin_time))
        if world > 1 and flags.check_pull:  # synchronous replicas: identical parameters on every worker
            log("params checksum %.12e" % float(prog.P.master.double().sum().item()))
        if model.name in ("lstm", "cnn"):  # every worker evaluates and prints, as LSTM:134-138
            test_len = 128
            acc = prog.evaluate(torch.from_numpy(data.test.images[:test_len]).to(device),
                                torch.from_numpy(data.test.labels[:test_len]).to(device))
            log("Test-Accuracy: %2.4f" % acc)
    finally:
        if wd is not None:
            wd.stop()
        if hb is not None:
            hb.stop()
        if timer is not None:
            timer.close()
        sv.stop()
    return prog, opts, gstep


def _leave_watchdog(store, rank, world, timeout_s):
    """End of training with the comm watchdog on: the TCPStore lives in rank 0's process, so rank 0
    waits (bounded) until every rank has stopped its watchdog before it can exit - a peer still
    polling would otherwise read the vanished store as a failure.
    The counter is never reset: a store reused by a later run (tests, an in-process rerun) keeps
    counting, and each rank's own ticket tells which run it belongs to - every rank adds exactly
    once per run and a run cannot start before all ranks left the previous one - so rank 0 waits
    for the end of ITS run's group of `world` tickets."""
    key = "dtfe/hb/watchdogs_stopped"
    ticket = store.add(key, 1)
    if rank != 0:
        return
    target = ((ticket - 1) // world + 1) * world
    t_end = time.time() + timeout_s
    while store.add(key, 0) < target and time.time() < t_end:
        time.sleep(0.01)


def _ps_buckets(prog, bucket_mb=None):
    """Push buckets of a ps-mode worker: the program's own (the CNN's [head + fc1], [convs]) unless
    --bucket_mb is given, else ranges of the flat buffer, back to front."""
    core = getattr(prog, "core", None)
    if bucket_mb is None and core is not None and getattr(core, "buckets", None):
        return core.buckets
    return _buckets(prog.P, bucket_mb)


def _buckets(P, bucket_mb=None):
    """Contiguous gradient buckets of ``bucket_mb`` MB of fp32 gradient (default
    comm.DEFAULT_BUCKET_MB), back of the flat buffer first = backward-completion order."""
    from .parallel.comm import DEFAULT_BUCKET_MB

    mb = DEFAULT_BUCKET_MB if bucket_mb is None else float(bucket_mb)
    if mb <= 0:
        raise ValueError("--bucket_mb must be > 0")
    bucket_elems = max(1024, int(mb * (1 << 20)) // 4)
    total = P.total
    b = []
    hi = total
    while hi > 0:
        lo = max(0, hi - bucket_elems)
        b.append((lo, hi))
        hi = lo
    return b


# ------------------------------------------------------------------- entry
def run(model_name: str, argv=None, log=_print):
    cls, lr = MODELS[model_name]
    m0 = cls()
    flags = flagmod.parse(argv, model_defaults=dict(batch_size=m0.default_batch, num_steps=m0.default_steps,
                                                    learning_rate=lr), prog="distributed_%s.py" % model_name)
    model = cls(lr=flags.learning_rate)
    try:
        model.set_dtype(flags.dtype)  # --dtype: the model's program must implement it (no silent fallback)
    except ValueError as e:
        raise SystemExit(str(e))
    torch.manual_seed(flags.seed)
    np.random.seed(flags.seed)
    mode = flagmod.resolve_mode(flags)  # (+ mode-dependent defaults: --heartbeat_secs)
    local_rank = int(os.environ.get("LOCAL_RANK", flags.task_index if flags.job_name == "worker" else 0))
    device = resolve_device(flags.device, local_rank)
    if device.type == "cuda":
        torch.cuda.set_device(device)
    backend = resolve_backend(flags.backend, device)
    if mode == "local":
        run_allreduce(flags, model, device, log)
        return 0
    cluster = ClusterSpec.from_flags(flags.ps_hosts, flags.worker_hosts)
    if mode == "ps":
        if not cluster.ps:
            raise SystemExit("--mode=ps needs --ps_hosts")
        server = Server(cluster, flags.job_name, flags.task_index, backend=backend,
                        device=device if backend == "nccl" else None)
        try:
            if flags.job_name == "ps":
                run_ps(flags, model, server, device, log)
            elif flags.job_name == "worker":
                run_worker_ps(flags, model, server, device, log)
            else:
                raise SystemExit("--job_name must be 'ps' or 'worker'")
        finally:
            server.shutdown()
        return 0
    # ring all-reduce: workers only
    if flags.job_name == "ps":
        log("ps %d: nothing to serve in --mode=allreduce; quitting" % flags.task_index)
        return 0
    cluster = ClusterSpec([], cluster.worker)
    server = Server(cluster, "worker", flags.task_index, backend=backend,
                    device=device if backend == "nccl" else None)
    try:
        run_allreduce(flags, model, device, log, world=cluster.world_size, rank=server.rank, store=server.store)
    finally:
        server.shutdown()
    return 0


def main(model_name: str):
    sys.exit(run(model_name, sys.argv[1:]))
