#!/usr/bin/env python
"""Headline benchmark: MNIST 2-layer CNN, sync all-reduce data parallel, bf16,
images/sec for the whole job (BASELINE.json metric).

    python bench.py --gpus N --steps K --warmup W        (self-launches N ranks)
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...
    python bench.py --model resnet20 | resnet50          (BASELINE.json configs 3 and 5)
    python bench.py --mode ps --gpus N                   (config 4: 1 ps + N workers, async)

Launching: under torchrun (``WORLD_SIZE`` set) each process is one rank.  Without
``WORLD_SIZE`` and with ``--gpus N > 1`` this process is a pure launcher: it starts N
child ranks of itself (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 in their
environment) BEFORE touching the GPU, waits for them, and exits with the worst exit
code; rank 0's JSON line is the result.  Every rank asserts WORLD_SIZE == --gpus.

Weak scaling: every rank trains --batch_size images per step (global batch =
batch_size * N).  Synthetic MNIST-shaped data resident in HBM, random-init
weights.  Before the W warmup steps, --prewarm_ms (150) of training steps bring the
GPU clocks up (reported as config.prewarm; see timed()).  The timed region is exactly K full training steps (device-side batch
sampling, forward, backward, gradient all-reduce, fused Adam), bracketed by
barrier + device synchronize on both sides; the reported time is the MAX over
ranks.  The K steps are also cut into up to 5 windows by hipEvents recorded
between replays (no sync inside the timed region) so the JSON carries its own
spread.  Steps run as hipGraph replays of --steps_per_graph S consecutive steps
(default 4 on one GPU, 1 with several ranks; K is timed whatever S is, a remainder
runs as single-step replays, and both graphs are captured before the timed region -
those capture steps are counted in config.prewarm.steps).  Rank 0 prints one JSON line.

Reference: the reference's only performance output is its per-step wall-clock
print (gan/distributed_gan.py:195-196, encoder/distributed_encoder.py:166-167).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import torch  # noqa: E402  (importing torch does not initialise the GPU)
import torch.distributed as dist  # noqa: E402

DEFAULT_BATCH = 1024  # per GPU, MNIST CNN
MODEL_BATCH = {"mnist_cnn": 1024, "resnet20": 256, "resnet50": 256}


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None, help="number of ranks (one per GPU); default 1 "
                    "or WORLD_SIZE under torchrun")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--prewarm_ms", type=float, default=150.0,
                    help="before the W warmup steps, replay training steps for this long (GPU clock ramp; "
                         "reported as config.prewarm); 0 disables")
    ap.add_argument("--batch_size", type=int, default=None, help="per-GPU batch (default: per model)")
    ap.add_argument("--comm_dtype", choices=["fp32", "bf16"], default="bf16")
    ap.add_argument("--dtype", choices=["bf16", "fp32"], default="bf16",
                    help="compute dtype of the MNIST CNN: bf16 (the headline) or fp32 (the reference's precision: "
                         "exact-fp32 MFMA kernels, fp32 activations; one GPU)")
    ap.add_argument("--bucket_mb", type=float, default=None,
                    help="ResNet gradient bucket size, MB of fp32 gradient (default parallel.comm.DEFAULT_BUCKET_MB; "
                         "the CNN keeps its two buckets [head + fc1] / [convs])")
    ap.add_argument("--no_graph", action="store_true")
    ap.add_argument("--no_join_defer", action="store_true",
                    help="CNN: join the conv2 weight-gradient branch before Adam in every step (A/B hook)")
    ap.add_argument("--steps_per_graph", type=int, default=0,
                    help="training steps captured per hipGraph replay (TF2 steps_per_execution; every step is "
                         "still a full step, K steps are timed whatever S is).  0: 4 on one GPU, 1 with "
                         "several ranks")
    ap.add_argument("--model", choices=["mnist_cnn", "resnet20", "resnet50"], default="mnist_cnn")
    ap.add_argument("--mode", choices=["allreduce", "ps"], default="allreduce",
                    help="allreduce: sync data parallel (headline).  ps: async parameter server, "
                         "1 ps service + --gpus workers (BASELINE.json config 4)")
    ap.add_argument("--comm", choices=["auto", "rccl", "ipc", "pg"], default="auto",
                    help="auto: per bucket size the faster of dtfe's RCCL communicator and the hipIpc two-shot "
                         "kernel (timed at setup); rccl / ipc: force one; all three run on a side stream with the "
                         "whole step captured in one hipGraph.  pg: torch.distributed ProcessGroupNCCL, eager steps")
    ap.add_argument("--hogwild", action="store_true", help="--mode ps: lock-free concurrent applies")
    ap.add_argument("--ps_overlap", choices=["auto", "on", "off"], default="auto",
                    help="--mode ps: apply pushed buckets during backward (auto: only on a ps GPU other "
                         "than the worker's)")
    ap.add_argument("--ps_fused_reply", choices=["on", "off"], default="on",
                    help="--mode ps: async applies write the worker's reply buffer themselves (on) or the ps "
                         "copies a snapshot into it (off; tests compare the two bit for bit)")
    ap.add_argument("--ps_stream", default="normal",
                    help="--mode ps: the ps apply stream - normal, high (highest queue priority) or cu<N> (CU mask "
                         "of N CUs); the ps shares GPU 0 with worker 0")
    ap.add_argument("--num_ps", type=int, default=1,
                    help="--mode ps: ps tasks (P); ps k runs on GPU k * ndev / P (distinct GPUs when ndev >= P)")
    ap.add_argument("--ps_partition_mb", type=float, default=0.0,
                    help="--mode ps: partition variables larger than this many MB over the ps tasks "
                         "(parallel/partition.py; the CNN's fc1 weight is 12.8 MB)")
    ap.add_argument("--ps_verify", type=int, default=0, help=argparse.SUPPRESS)  # test hook, see bench_ps
    ap.add_argument("--backend", choices=["nccl", "gloo"], default="nccl",
                    help="nccl = RCCL (one rank per GPU); gloo only to rehearse several ranks on one GPU")
    return ap.parse_args(argv)


# ----------------------------------------------------------------------------- launcher
def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int, argv) -> int:
    """Start ``n`` child ranks of this script (no GPU call has been made in this process) and
    return the worst exit code.  If one rank fails the others are stopped (by PID)."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), DTFE_BENCH_CHILD="1")
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__)] + list(argv), env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            r = p.poll()
            if r is None:
                continue
            live.remove(p)
            if r != 0:
                rc = rc or r
                for q in live:  # a failed rank would leave its peers blocked in a collective
                    q.terminate()
        time.sleep(0.05)
    for p in procs:
        p.wait()
        if p.returncode not in (0, None) and rc == 0:
            rc = p.returncode
    return rc if rc >= 0 else 128 - rc


# ----------------------------------------------------------------------------- per rank
class Dist:
    def __init__(self, args):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        want = args.gpus if args.gpus is not None else self.world
        if want != self.world:
            raise SystemExit("bench.py: --gpus %d but WORLD_SIZE=%d" % (want, self.world))
        self.backend = args.backend
        if self.world > 1:
            ndev = torch.cuda.device_count()
            if args.backend == "nccl" and self.local_rank >= ndev:
                raise SystemExit("bench.py: rank %d needs GPU %d but only %d are visible (RCCL needs one GPU "
                                 "per rank; use --backend gloo --comm ipc to rehearse on fewer GPUs)"
                                 % (self.rank, self.local_rank, ndev))
            self.local_rank %= max(1, ndev)
            torch.cuda.set_device(self.local_rank)
            if args.backend == "nccl":
                dist.init_process_group("nccl", device_id=torch.device("cuda", self.local_rank))
            else:
                dist.init_process_group("gloo")
        self.device = torch.device("cuda", self.local_rank)

    def barrier(self):
        if self.world > 1:
            dist.barrier()

    def max(self, x: float) -> float:
        if self.world == 1:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=self.device if self.backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def distinct_devices(self) -> int:
        """Distinct physical GPUs behind the ranks (a gloo rehearsal may share one)."""
        me = "%s:%d" % (socket.gethostname(), self.local_rank)
        if self.world == 1:
            return 1
        allv = [None] * self.world
        dist.all_gather_object(allv, me)
        return len(set(allv))

    def close(self):
        if self.world > 1:
            dist.destroy_process_group()


def replicas_identical(params, d: Dist):
    """After the timed steps (outside the timing): every replica trained on different data
    but applied the same all-reduced gradients, so all parameter copies must be bitwise equal."""
    ref = params.detach().clone() if d.backend == "nccl" else params.detach().cpu()
    dist.broadcast(ref, src=0)
    diff = (params.detach().to(ref.device) - ref).abs().max().reshape(1).double()
    dist.all_reduce(diff, op=dist.ReduceOp.MAX)
    return bool(float(diff.item()) == 0.0)


def _steps_per_graph(args, d) -> int:
    """Training steps per hipGraph replay: --steps_per_graph, else 4 on one GPU (the graph-launch gap
    between replays is ~1.5 % of a CNN step: 0.1923-0.1933 -> 0.1903-0.1904 ms, profiles/r6_steps_per_graph.txt)
    and 1 with several ranks (their captured collectives are only rehearsed on one GPU here)."""
    if args.steps_per_graph > 0:
        return args.steps_per_graph
    return 4 if d.world == 1 else 1


def timed(runner, steps: int, warmup: int, d: Dist, prewarm_ms: float = 0.0):
    """Pre-warm, W untimed steps, then exactly K steps between barrier+sync brackets.  Returns
    (elapsed_s max over ranks, per-window ms/step list measured on this rank, pre-warm steps).

    Pre-warm: full training steps, replayed in chunks of 10 until ``prewarm_ms`` have passed
    (the rank-max elapsed time decides, so every rank runs the same steps).  An idle MI355X
    ramps its clocks over the first tens of ms of load: with the driver's W=5 / K=20 CNN run
    (1 + 4 ms of GPU work) the timed windows fell from 0.212 to 0.204 ms/step, after 100
    untimed steps they sat at 0.195-0.196 (profiles/r4_cnn_clock_ramp.txt).  The pre-warm
    steps are real steps (they train the model) and are reported in the JSON config."""
    run = runner.run if hasattr(runner, "run") else (lambda n: [runner() for _ in range(n)])
    S = getattr(runner, "steps", 1)
    pre = 0
    if prewarm_ms > 0:
        t = time.perf_counter()
        chunk = max(10, S)
        while True:
            run(chunk)
            pre += chunk
            torch.cuda.synchronize()
            if d.max(time.perf_counter() - t) * 1000.0 >= prewarm_ms:
                break
    if hasattr(runner, "prime"):  # graph captures happen here, never inside the timed steps
        pre += runner.prime()
    run(warmup)
    torch.cuda.synchronize()
    d.barrier()
    torch.cuda.synchronize()
    nwin = max(1, min(5, steps))
    # window cuts on replay boundaries (multiples of the steps per replay), the last one at K
    cuts = sorted(set([0] + [min(steps, round(i * steps / nwin / S) * S) for i in range(1, nwin)] + [steps]))
    nwin = len(cuts) - 1
    evs = [torch.cuda.Event(enable_timing=True) for _ in cuts]
    t0 = time.perf_counter()
    evs[0].record()
    for w in range(nwin):
        run(cuts[w + 1] - cuts[w])
        evs[w + 1].record()
    torch.cuda.synchronize()
    d.barrier()
    torch.cuda.synchronize()
    elapsed = d.max(time.perf_counter() - t0)
    win = [evs[i].elapsed_time(evs[i + 1]) / max(1, cuts[i + 1] - cuts[i]) for i in range(nwin)]
    return elapsed, win, pre


def _baseline(n_gpus, batch, model="mnist_cnn"):
    """Faster of the stock-PyTorch rows (eager DDP; graph-captured + fused Adam/SGD) measured on
    the same MI355X and config by bench/stock_torch_cnn.py / stock_torch_resnet.py.
    Without a measured N-GPU stock row the bar is N x the best 1-GPU stock row (stock with ideal
    scaling - never easier than the real stock DDP curve)."""
    p = os.path.join(ROOT, "bench", "stock_baseline.json")
    try:
        with open(p) as f:
            tab = json.load(f)
    except (OSError, ValueError):
        return None

    def best(n):
        key = f"{n}x{batch}" if model == "mnist_cnn" else f"{model}_{n}x{batch}"
        vals = [v for k, v in tab.items() if (k == key or k.startswith(key + "_")) and isinstance(v, (int, float))]
        return max(vals) if vals else None

    b = best(n_gpus)
    if b is None and n_gpus > 1 and best(1) is not None:
        b = n_gpus * best(1)
    return b


def _make_comm(args, d: Dist, bucket_bytes):
    from dtfe.parallel.comm import make_comm

    if d.world == 1 or args.comm == "pg" or not (args.backend == "nccl" or args.comm == "ipc"):
        return None
    return make_comm(d.device, None, bucket_bytes,
                     torch.bfloat16 if args.comm_dtype == "bf16" else torch.float32, mode=args.comm,
                     log=(lambda m: print(m, file=sys.stderr, flush=True)) if d.rank == 0 else None)


def _comm_info(args, d: Dist, comm):
    if d.world == 1:
        return {"grad_allreduce": "none (1 rank)", "ranks_seen_by_comm": 1}
    if comm is not None:
        eng = "in-graph [%s]" % comm.describe()
        seen = comm.world
    else:
        eng = "ProcessGroupNCCL (RCCL)" if args.backend == "nccl" else "gloo"
        seen = dist.get_world_size()
    return {"grad_allreduce": "%s bucketed %s" % (eng, args.comm_dtype), "ranks_seen_by_comm": seen}


def _emit(d: Dist, args, metric, value, elapsed, win, model_desc, B, extra, data_desc):
    # (the stock baseline rows are bf16; an fp32 run is compared in BASELINE.md against the stock fp32 row)
    base = _baseline(d.world, B, args.model) if getattr(args, "dtype", "bf16") == "bf16" else None
    rec = {
        "metric": metric,
        "value": round(value, 1),
        "unit": "images/sec",
        "n_gpus": d.world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1000, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": round(value / base, 3) if base else None,
        "dtype": getattr(args, "dtype", "bf16"),
        "data": data_desc,
        "config": dict({"model": model_desc, "global_batch": B * d.world, "seq_len": None,
                        "parallelism": "dp%d" % d.world, "per_gpu_batch": B}, **extra),
        "window_ms_per_step": [round(x, 4) for x in win],
        "median_window_ms_per_step": round(statistics.median(win), 4),
    }
    if d.rank == 0:
        print(json.dumps(rec), flush=True)


def bench_cnn(args, d: Dist):
    import dtfe  # noqa: F401
    from dtfe.models.mnist_cnn import MnistCnnTrainer, num_params
    from dtfe.parallel.allreduce import BucketAllReduce
    from dtfe.utils.graphs import MultiStepGraph, graphs_enabled

    B = args.batch_size or MODEL_BATCH["mnist_cnn"]
    if args.dtype == "fp32":
        from dtfe.models.mnist_cnn import MnistCnnF32Trainer
        if d.world != 1:
            raise SystemExit("bench.py --dtype fp32: one GPU (the reference-precision row)")
        trainer = MnistCnnF32Trainer(B, d.device, seed=0)
    else:
        trainer = MnistCnnTrainer(B, d.device, seed=0, world_size=d.world, rank=d.rank)
    comm = allreduce = None
    cdt = torch.bfloat16 if args.comm_dtype == "bf16" else torch.float32
    if d.world > 1:
        esz = 2 if args.comm_dtype == "bf16" else 4
        comm = _make_comm(args, d, [(hi - lo) * esz for lo, hi in trainer.buckets])
        allreduce = BucketAllReduce(trainer.P.grad, trainer.buckets, comm=comm, comm_dtype=cdt)
        trainer.allreduce = allreduce

    if allreduce is not None and allreduce.grad16 is not None:
        def step():
            trainer.step(grad16=allreduce.grad16, gscale=1.0 / d.world)
    else:
        step = trainer.step
    # the whole step (with the overlapped all-reduce at world > 1) is one hipGraph replay
    spg = _steps_per_graph(args, d)
    # one replica, several steps per replay: the conv2 weight-gradient branch rejoins once per replay and
    # signals Adam on the device instead (MnistCnnTrainer.defer_join; profiles/r6_steps_per_graph.txt)
    trainer.defer_join = spg > 1 and allreduce is None and args.dtype != "fp32" and not args.no_join_defer
    runner = MultiStepGraph(step, spg, warmup=2,
                            enabled=((d.world == 1 or comm is not None) and not args.no_graph and graphs_enabled()),
                            capture_error_mode="thread_local", finish=trainer.join_side)
    elapsed, win, pre = timed(runner, args.steps, args.warmup, d, args.prewarm_ms)
    if comm is not None and hasattr(comm, "check_health"):
        comm.check_health()
    loss = float(trainer.loss_sum.item()) / B
    same = replicas_identical(trainer.P.master, d) if d.world > 1 else None
    ndev = d.distinct_devices()
    extra = {"optimizer": "adam (TF1)", "hip_graph": runner.graph is not None, "steps_per_graph": runner.steps,
             "join_deferred": bool(getattr(trainer, "defer_join", False)), "last_loss": round(loss, 4),
             "replicas_identical": same, "distinct_gpus": ndev, "prewarm": {"ms": args.prewarm_ms, "steps": pre}}
    extra.update(_comm_info(args, d, comm))
    _emit(d, args, "images/sec (whole node), MNIST CNN sync all-reduce", B * d.world * args.steps / elapsed,
          elapsed, win, "mnist_cnn (conv5x5x32-pool-conv5x5x64-pool-fc1024-dropout-fc10, %d params)" % num_params(),
          B, extra, "synthetic (HBM-resident MNIST-shaped uint8 images, random labels; random-init weights)")
    if comm is not None:
        comm.close()


def bench_resnet(args, d: Dist):
    """ResNet-20 (CIFAR-10 shape) / ResNet-50 (ImageNet shape) sync all-reduce step: device-side
    batch sampling (+ one-hot labels) from an HBM-resident synthetic set, fwd+bwd, all-reduce,
    Momentum apply."""
    import dtfe  # noqa: F401
    from dtfe import ops
    from dtfe.models.resnet import ResNetModel
    from dtfe.optim import Optimizer
    from dtfe.parallel.allreduce import BucketAllReduce
    from dtfe.train import _buckets
    from dtfe.utils.graphs import MultiStepGraph, graphs_enabled

    model = ResNetModel(arch=args.model)
    B = args.batch_size or MODEL_BATCH[args.model]
    prog = model.program(d.device, B, seed=0)
    gstep = torch.zeros(1, dtype=torch.int32, device=d.device)
    cfg, names, bp = model.opt_groups[0]
    opt = Optimizer(cfg, prog.P, var_list=names, global_step=gstep, beta_power_names=bp)
    ar = comm = None
    cdt = torch.bfloat16 if args.comm_dtype == "bf16" else torch.float32
    if d.world > 1:
        if d.backend == "nccl":
            dist.broadcast(prog.P.master, src=0)
        else:
            m = prog.P.master.detach().cpu()
            dist.broadcast(m, src=0)
            prog.P.master.copy_(m)
        prog.P.refresh_copies()
        bks = _buckets(prog.P, args.bucket_mb)
        esz = 2 if args.comm_dtype == "bf16" else 4
        comm = _make_comm(args, d, [(hi - lo) * esz for lo, hi in bks])
        ar = BucketAllReduce(prog.P.grad, bks, comm=comm, comm_dtype=cdt)
        prog.grad_ready = ar.ready  # buckets launch during backward (overlap on the side stream)
    n_pool = 4096 if args.model == "resnet20" else 512
    g = torch.Generator().manual_seed(d.rank + 11)
    pix = model.image * model.image * model.channels
    images = torch.randint(0, 256, (n_pool, pix), generator=g, dtype=torch.uint8).to(d.device)
    labels = torch.randint(0, model.num_classes, (n_pool,), generator=g, dtype=torch.int32).to(d.device)
    lab = torch.empty(B, dtype=torch.int32, device=d.device)
    ctr = torch.zeros(1, dtype=torch.int64, device=d.device)
    done = torch.zeros(1, dtype=torch.int32, device=d.device)

    def step():
        # batch rows + their one-hot label rows in ONE launch (no per-step fill / scatter kernels)
        ops.gather_rows(images, prog.x.view(B, -1), None, labels, lab, seed=d.rank + 1, counter=ctr, done=done,
                        zero=prog.step_accumulators(), onehot=prog.y)
        prog.compute_grads(zeroed=True)
        g16 = None
        if ar is not None:
            ar.flush()
            ar.wait()
            g16 = ar.grad16
        opt.step(grad16=g16, gscale=1.0 / d.world) if g16 is not None else opt.step(gscale=1.0 / d.world)

    runner = MultiStepGraph(step, _steps_per_graph(args, d), warmup=2, enabled=((d.world == 1 or comm is not None) and not args.no_graph
                                                and graphs_enabled()), capture_error_mode="thread_local")
    elapsed, win, pre = timed(runner, args.steps, args.warmup, d, args.prewarm_ms)
    # trainable variables only: BN moving statistics are per-replica (each rank's own batches)
    train_vals = torch.cat([prog.P.view(n).reshape(-1) for n in names])
    same = replicas_identical(train_vals, d) if d.world > 1 else None
    extra = {"optimizer": "momentum 0.9 (TF1)", "hip_graph": runner.graph is not None, "steps_per_graph": runner.steps,
             "last_loss": round(float(prog.loss.item()) / B, 4), "replicas_identical": same,
             "distinct_gpus": d.distinct_devices(), "prewarm": {"ms": args.prewarm_ms, "steps": pre}}
    extra.update(_comm_info(args, d, comm))
    _emit(d, args, "images/sec (whole node), %s sync all-reduce" % args.model, B * d.world * args.steps / elapsed,
          elapsed, win, "%s (%d params)" % (args.model, model.num_params()), B, extra,
          "synthetic (HBM-resident %dx%dx%d uint8 images, random labels; random-init weights)"
          % (model.image, model.image, model.channels))
    if comm is not None:
        comm.close()


def bench_ps(args):
    """BASELINE.json config 4: MNIST CNN async parameter-server SGD, P ps + N workers on one node.

    Ranks 0..P-1 are the ps tasks (each its round-robin shard of the variables + their TF1 Adam slots,
    ps k on GPU k * ndev / P, served by the native C++ progress thread of ``parallel/ps_native.py``;
    with --ps_partition_mb the fc1 weight is split into partitions dealt over the ps tasks,
    parallel/partition.py); ranks P..P+N-1 are workers on GPUs 0..N-1.  A worker step = HBM batch sampling fused into conv1, forward, backward with the
    gradient buckets pushed into the ps's hipIpc mailboxes on a side stream while backward
    continues (bf16 over xGMI), a device-side request / wait for the ps's apply, and the pull of
    the fresh bf16 working copies - one hipGraph replay, no host round trip.  Every push is
    applied (async: one at a time in arrival order; --hogwild: concurrently).  Timed: K steps
    per worker between worker barriers + device syncs, MAX over workers; images/sec counts
    every worker's images.  Reference: gan/distributed_gan.py:119-121,193 (push/pull per
    sess.run), :195-196 (its per-step timing print)."""
    import dtfe  # noqa: F401
    from dtfe.models.mnist_cnn import MnistCnnModel, MnistCnnTrainer, num_params
    from dtfe.parallel import ps_native
    from dtfe.parallel.cluster import ClusterSpec, Server
    from dtfe.parallel.ps import PSClient, PSServer, Shard, wait_for_init
    from dtfe.parallel.partition import PartitionedModel
    from dtfe.train import _shard_layout
    from dtfe.utils.graphs import StepGraph, graphs_enabled

    N, NP = args.gpus or 1, max(1, args.num_ps)
    world, rank = int(os.environ["WORLD_SIZE"]), int(os.environ["RANK"])
    if world != N + NP:
        raise SystemExit("bench.py --mode ps: expected %d processes (%d ps + %d workers), got %d"
                         % (N + NP, NP, N, world))
    ndev = max(1, torch.cuda.device_count())
    port = int(os.environ["MASTER_PORT"])
    cluster = ClusterSpec(["127.0.0.1:%d" % (port + i) for i in range(NP)],
                          ["127.0.0.1:%d" % (port + NP + i) for i in range(N)])
    job, idx = cluster.task_of(rank)
    gpu = (idx * ndev // NP) % ndev if job == "ps" else idx % ndev
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    server = Server(cluster, job, idx, backend="nccl", device=dev)
    full_model = MnistCnnModel()
    model = PartitionedModel(full_model, int(args.ps_partition_mb * (1 << 20))) if args.ps_partition_mb > 0 \
        else full_model
    placement, shard_specs = _shard_layout(model, NP)
    gs_ps = placement[model.gs_name]
    B = args.batch_size or MODEL_BATCH["mnist_cnn"]
    if job == "ps":
        shard = Shard(shard_specs[idx], model.opt_groups, dev, gs_ps == idx, model.gs_increments)
        ps = PSServer(server, shard, num_workers=N, comm_device="cpu", log=lambda *_: None)
        ps.native = ps_native.NativeShardService(server, shard, N, hogwild=args.hogwild,
                                                 fused_replies=args.ps_fused_reply == "on", stream=args.ps_stream)
        ps.serve_forever()
        st = ps.native.stats()
        ps.native.stop()
        server.store.set("dtfe/bench/ps_stats/%d" % idx, json.dumps(dict(st, global_step=shard.global_step(),
                                                                         numel=shard.numel, gpu=gpu)))
        print("ps %d: %s" % (idx, json.dumps(st)), file=sys.stderr, flush=True)
        server.shutdown()
        _rank_exit()

    def wsum(x: float, op=dist.ReduceOp.SUM) -> float:
        t = torch.tensor([x], dtype=torch.float64)  # CPU tensor: the gloo half of the worker group
        dist.all_reduce(t, op=op, group=server.worker_group)
        return float(t.item())

    tr = MnistCnnTrainer(B, dev, seed=0, rank=idx)
    if isinstance(model, PartitionedModel):
        model.add_aliases(tr.P)   # partitions as views of the worker's full variables
    client = PSClient(server, tr.P, placement, shard_specs, cluster.rank_of("ps", gs_ps), model.opt_groups,
                      comm_device="cpu")
    if idx == 0:
        client.init_variables()   # the chief's global_variables_initializer
    else:
        wait_for_init(client, poll_s=0.05)
    link = ps_native.NativePSLink(server, tr.P, placement, shard_specs, gs_ps, dev,
                                  buckets=tr.buckets, overlap={"auto": None, "on": True, "off": False}[args.ps_overlap])
    tr.allreduce = link           # bucket pushes fork off backward (MnistCnnTrainer.forward_backward)
    link.pull()

    def step():
        tr.forward_backward()
        link.end_step()

    runner = StepGraph(step, warmup=2, enabled=not args.no_graph and graphs_enabled(),
                       capture_error_mode="thread_local")

    def run1():
        runner()
        link.note_request()

    class _D:  # the timed() bracket over the workers only (the ps is serving)
        world = N

        @staticmethod
        def barrier():
            wsum(0.0)

        @staticmethod
        def max(x):
            return wsum(x, dist.ReduceOp.MAX)

    if args.ps_verify:
        _ps_verify(args, run1, link, client, tr, shard_specs, dev, server)

    elapsed, win, pre = timed(run1, args.steps, args.warmup, _D, args.prewarm_ms)
    gs = link.host_reply()
    link.check()
    loss = float(tr.loss_sum.item()) / B
    link.close()
    client.done()
    allst = [json.loads(server.store.get("dtfe/bench/ps_stats/%d" % k).decode()) for k in range(NP)] \
        if idx == 0 else None
    if idx == 0:
        stats = allst[gs_ps]
        pushes = N * (args.steps + args.warmup + pre)  # every runner() call is exactly one step (one push)
        rec_extra = {"optimizer": "adam (TF1), applied on the ps", "hip_graph": runner.graph is not None,
                     "last_loss": round(loss, 4), "global_step": gs, "ps_applies": stats.get("applies"),
                     "ps_bucket_applies": stats.get("bucket_applies"),
                     "ps_refreshed_ranges": stats.get("refreshed_ranges"),
                     "ps_global_step": stats.get("global_step"),
                     "pushes_issued": pushes, "ps_stream": args.ps_stream, "transport": "hipIpc mailboxes + C++ ps service (bf16 push, bf16 pull)",
                     "hogwild": bool(args.hogwild), "distinct_gpus": min(N, ndev), "ps_gpu": allst[0]["gpu"],
                     "num_ps": NP, "ps_partition_mb": args.ps_partition_mb,
                     "ps_shards": [{"gpu": a["gpu"], "params": a["numel"], "applies": a["applies"]} for a in allst],
                     "prewarm": {"ms": args.prewarm_ms, "steps": pre}}

        class _R:
            rank = 0
            world = N
        args_ps = argparse.Namespace(**vars(args))
        args_ps.model = "mnist_cnn_ps"
        _emit(_R, args_ps, "images/sec (whole node), MNIST CNN async parameter server (%d ps + %d workers)" % (NP, N),
              B * N * args.steps / elapsed, elapsed, win,
              "mnist_cnn (conv5x5x32-pool-conv5x5x64-pool-fc1024-dropout-fc10, %d params)" % num_params(), B,
              dict(rec_extra, parallelism="ps%d+w%d" % (NP, N)),
              "synthetic (HBM-resident MNIST-shaped uint8 images, random labels; random-init weights)")
    _rank_exit()


def _ps_verify(args, run1, link, client, tr, shard_specs, dev, server):
    """--ps_verify K (P ps + 1 worker, a test hook): K replayed worker steps; after each, the pulled
    bf16 working copies (natural + transposed) and fp32 variables must equal, bit for bit, what the
    ps shards' fp32 variables give (partitions compared as the worker's alias views) (fetched over the control channel while the ps is idle - one
    worker, its push applied).  Prints one JSON line with the per-step digests of the pulled copies
    (other data-plane variants must reproduce them) and exits."""
    import hashlib

    from dtfe.optim import FlatParams

    assert args.gpus in (None, 1), "--ps_verify: P ps + 1 worker"
    refs = {k: FlatParams(specs, dev, init=False) for k, specs in shard_specs.items() if specs}
    digests, mismatches = [], []
    for i in range(args.ps_verify):
        run1()
        link.host_reply()
        torch.cuda.synchronize()
        link.check()
        st, _gs = client.fetch_state()
        h = hashlib.sha1()
        for k, ref in sorted(refs.items()):
            ref.master.copy_(st[k][:ref.total].to(dev))
            ref.refresh_copies()
            for sp in shard_specs[k]:
                parts = []
                if sp.name in ref.w16:
                    parts.append(("w16", tr.P.w16[sp.name], ref.w16[sp.name]))
                if sp.name in ref.wt16:
                    parts.append(("wt16", tr.P.wt16[sp.name], ref.wt16[sp.name]))
                if not parts:
                    parts.append(("master", tr.P.view(sp.name), ref.view(sp.name)))
                for part, got, want in parts:
                    g = got.contiguous().view(-1).view(torch.int16 if got.dtype == torch.bfloat16 else torch.int32)
                    w = want.contiguous().view(-1).view(g.dtype)
                    if not torch.equal(g, w):
                        mismatches.append({"step": i, "var": sp.name, "part": part,
                                           "n_diff": int((g != w).sum().item())})
                    h.update(g.cpu().numpy().tobytes())
        digests.append(h.hexdigest()[:16])
    print(json.dumps({"ps_verify": digests, "mismatches": mismatches[:20], "n_mismatch": len(mismatches),
                      "fused_reply": args.ps_fused_reply, "overlap": args.ps_overlap}), flush=True)
    link.close()
    client.done()
    _rank_exit()


def _rank_exit() -> None:
    """End a ps-mode rank.  os._exit skips interpreter teardown (the peer-mapped mailboxes and the
    ps service thread need no orderly unwinding); DTFE_PROFILE_EXIT=1 exits normally instead so a
    profiler's exit handlers (rocprofv3 writes its trace at exit) run in every rank."""
    sys.stdout.flush()
    sys.stderr.flush()
    if os.environ.get("DTFE_PROFILE_EXIT") == "1":
        torch.cuda.synchronize()
        sys.exit(0)
    os._exit(0)


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse_args(argv)
    if args.mode == "ps":
        if os.environ.get("DTFE_BENCH_CHILD") != "1":
            # P ps + N workers = N + P processes on N GPUs (ps k shares GPU k * N / P with a worker)
            return launch_ranks((args.gpus or 1) + max(1, args.num_ps), argv)
        return bench_ps(args)
    if "WORLD_SIZE" not in os.environ and (args.gpus or 1) > 1:
        return launch_ranks(args.gpus, argv)
    d = Dist(args)
    try:
        if args.model == "mnist_cnn":
            bench_cnn(args, d)
        else:
            bench_resnet(args, d)
    finally:
        d.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
