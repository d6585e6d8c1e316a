#!/usr/bin/env python
"""Headline benchmark: MNIST 2-layer CNN, sync all-reduce data parallel, bf16,
images/sec for the whole job (BASELINE.json metric).

    python bench.py --gpus N --steps K --warmup W
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...
    python bench.py --model resnet20 | resnet50     (BASELINE.json configs 3 and 5)

Weak scaling: every rank trains --batch_size images per step (global batch =
batch_size * N).  Synthetic MNIST-shaped data resident in HBM, random-init
weights.  The timed region is exactly K full training steps (device-side batch
sampling, forward, backward, RCCL gradient all-reduce, fused Adam), bracketed
by barrier + device synchronize on both sides; the reported time is the MAX
over ranks.  Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import dtfe  # noqa: E402,F401
from dtfe.models.mnist_cnn import MnistCnnTrainer, num_params  # noqa: E402
from dtfe.parallel.allreduce import BucketAllReduce  # noqa: E402
from dtfe.parallel.comm import make_comm  # noqa: E402
from dtfe.utils.graphs import StepGraph, graphs_enabled  # noqa: E402

DEFAULT_BATCH = 1024  # per GPU


def _baseline(n_gpus, batch, model="mnist_cnn"):
    """Stock-PyTorch (DDP + MIOpen/hipBLASLt, bf16) images/sec measured on the same MI355X
    box and config by bench/stock_torch_cnn.py (bench/stock_torch_resnet.py for the
    ResNets); see BASELINE.md."""
    p = os.path.join(ROOT, "bench", "stock_baseline.json")
    try:
        with open(p) as f:
            tab = json.load(f)
        key = f"{n_gpus}x{batch}" if model == "mnist_cnn" else f"{model}_{n_gpus}x{batch}"
        return tab.get(key)
    except (OSError, ValueError):
        return None


def replicas_identical(params, device, backend):
    """After the timed steps (outside the timing): every replica trained on different data
    but applied the same all-reduced gradients, so all parameter copies must be bitwise equal."""
    ref = params.detach().clone() if backend == "nccl" else params.detach().cpu()
    dist.broadcast(ref, src=0)
    d = (params.detach().to(ref.device) - ref).abs().max().reshape(1).double()
    dist.all_reduce(d, op=dist.ReduceOp.MAX)
    return bool(float(d.item()) == 0.0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch_size", type=int, default=DEFAULT_BATCH, help="per-GPU batch")
    ap.add_argument("--comm_dtype", choices=["fp32", "bf16"], default="bf16")
    ap.add_argument("--no_graph", action="store_true")
    ap.add_argument("--model", choices=["mnist_cnn", "resnet20", "resnet50"], default="mnist_cnn")
    ap.add_argument("--comm", choices=["auto", "rccl", "ipc", "pg"], default="auto",
                    help="auto: per bucket size the faster of dtfe's RCCL communicator and the hipIpc two-shot "
                         "kernel (timed at setup); rccl / ipc: force one; all three run on a side stream with the "
                         "whole step captured in one hipGraph.  pg: torch.distributed ProcessGroupNCCL, eager steps")
    ap.add_argument("--backend", choices=["nccl", "gloo"], default="nccl",
                    help="nccl = RCCL (one rank per GPU); gloo only to rehearse several ranks on one GPU")
    args = ap.parse_args()
    if args.model != "mnist_cnn":
        return bench_resnet(args)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        local_rank %= torch.cuda.device_count()
        torch.cuda.set_device(local_rank)
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        else:
            dist.init_process_group("gloo")
    device = torch.device("cuda", local_rank)

    allreduce = None
    trainer = MnistCnnTrainer(args.batch_size, device, seed=0, world_size=world, rank=rank)
    comm = None
    if world > 1:
        if args.comm != "pg" and (args.backend == "nccl" or args.comm == "ipc"):
            esz = 2 if args.comm_dtype == "bf16" else 4
            comm = make_comm(device, None, [(hi - lo) * esz for lo, hi in trainer.buckets],
                             torch.bfloat16 if args.comm_dtype == "bf16" else torch.float32, mode=args.comm,
                             log=(lambda m: print(m, file=sys.stderr, flush=True)) if rank == 0 else None)
        allreduce = BucketAllReduce(trainer.P.grad, trainer.buckets, comm=comm,
                                    comm_dtype=torch.bfloat16 if args.comm_dtype == "bf16" else torch.float32)
        trainer.allreduce = allreduce

    if allreduce is not None and allreduce.grad16 is not None:
        def step():
            trainer.step(grad16=allreduce.grad16, gscale=1.0 / world)
    else:
        step = trainer.step
    # the whole step (with the overlapped RCCL all-reduce at world > 1) is one hipGraph replay
    runner = StepGraph(step, warmup=2, enabled=((world == 1 or comm is not None) and not args.no_graph
                                                and graphs_enabled()), capture_error_mode="thread_local")

    for _ in range(args.warmup):
        runner()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        runner()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=device if args.backend == "nccl" else "cpu", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    loss = float(trainer.loss_sum.item()) / args.batch_size
    consistent = replicas_identical(trainer.P.master, device, args.backend) if world > 1 else None
    global_batch = args.batch_size * world
    value = global_batch * args.steps / elapsed
    base = _baseline(world, args.batch_size)
    if rank == 0:
        print(json.dumps({
            "metric": "images/sec (whole node), MNIST CNN sync all-reduce",
            "value": round(value, 1),
            "unit": "images/sec",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1000, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(value / base, 3) if base else None,
            "dtype": "bf16",
            "data": "synthetic (HBM-resident MNIST-shaped uint8 images, random labels; random-init weights)",
            "config": {
                "model": "mnist_cnn (conv5x5x32-pool-conv5x5x64-pool-fc1024-dropout-fc10, %d params)" % num_params(),
                "global_batch": global_batch,
                "seq_len": None,
                "parallelism": "dp%d" % world,
                "per_gpu_batch": args.batch_size,
                "optimizer": "adam (TF1)",
                "grad_allreduce": ("%s bucketed %s" % ("in-graph [%s]" % comm.describe() if comm is not None else
                                                       "rccl (ProcessGroupNCCL)" if args.backend == "nccl" else "gloo",
                                                       args.comm_dtype))
                if world > 1 else "none (1 rank)",
                "hip_graph": runner.graph is not None,
                "last_loss": round(loss, 4),
                "replicas_identical": consistent,
            },
        }), flush=True)
    if world > 1:
        dist.destroy_process_group()


def bench_resnet(args):
    """ResNet-20 (CIFAR-10 shape) / ResNet-50 (ImageNet shape) sync all-reduce step: device-side
    batch sampling from an HBM-resident synthetic set, fwd+bwd, RCCL all-reduce, Momentum apply."""
    from dtfe import ops
    from dtfe.models.resnet import ResNetModel
    from dtfe.optim import Optimizer
    from dtfe.train import _buckets

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    device = torch.device("cuda", local_rank)
    model = ResNetModel(arch=args.model)
    B = args.batch_size if args.batch_size != DEFAULT_BATCH else (256 if args.model == "resnet20" else 64)
    prog = model.program(device, B, seed=0)
    gstep = torch.zeros(1, dtype=torch.int32, device=device)
    cfg, names, bp = model.opt_groups[0]
    opt = Optimizer(cfg, prog.P, var_list=names, global_step=gstep, beta_power_names=bp)
    ar = comm = None
    if world > 1:
        dist.broadcast(prog.P.master, src=0)
        prog.P.refresh_copies()
        bks = _buckets(prog.P)
        esz = 2 if args.comm_dtype == "bf16" else 4
        comm = make_comm(device, None, [(hi - lo) * esz for lo, hi in bks],
                         torch.bfloat16 if args.comm_dtype == "bf16" else torch.float32, mode=args.comm,
                         log=(lambda m: print(m, file=sys.stderr, flush=True)) if rank == 0 else None) \
            if args.comm != "pg" else None
        ar = BucketAllReduce(prog.P.grad, bks, comm=comm,
                             comm_dtype=torch.bfloat16 if args.comm_dtype == "bf16" else torch.float32)
        prog.grad_ready = ar.ready  # buckets launch during backward (overlap on RCCL's stream)
    n_pool = 4096 if args.model == "resnet20" else 512
    g = torch.Generator().manual_seed(rank + 11)
    pix = model.image * model.image * model.channels
    images = torch.randint(0, 256, (n_pool, pix), generator=g, dtype=torch.uint8).to(device)
    labels = torch.randint(0, model.num_classes, (n_pool,), generator=g, dtype=torch.int32).to(device)
    lab = torch.empty(B, dtype=torch.int32, device=device)
    ctr = torch.zeros(1, dtype=torch.int64, device=device)
    done = torch.zeros(1, dtype=torch.int32, device=device)

    def step():
        ops.gather_rows(images, prog.x.view(B, -1), None, labels, lab, seed=rank + 1, counter=ctr, done=done)
        prog.y.zero_()
        prog.y.scatter_(1, lab.long().unsqueeze(1), 1.0)
        prog.compute_grads()
        g16 = None
        if ar is not None:
            ar.flush()
            ar.wait()
            g16 = ar.grad16
        opt.step(grad16=g16, gscale=1.0 / world) if g16 is not None else opt.step(gscale=1.0 / world)

    runner = StepGraph(step, warmup=2, enabled=((world == 1 or comm is not None) and not args.no_graph
                                                and graphs_enabled()), capture_error_mode="thread_local")
    for _ in range(args.warmup):
        runner()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        runner()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    value = B * world * args.steps / elapsed
    base = _baseline(world, B, args.model)
    if rank == 0:
        print(json.dumps({
            "metric": "images/sec (whole node), %s sync all-reduce" % args.model,
            "value": round(value, 1), "unit": "images/sec", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1000, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": round(value / base, 3) if base else None, "dtype": "bf16",
            "data": "synthetic (HBM-resident %dx%dx%d uint8 images, random labels; random-init weights)"
                    % (model.image, model.image, model.channels),
            "config": {"model": "%s (%d params)" % (args.model, model.num_params()), "global_batch": B * world,
                       "seq_len": None, "parallelism": "dp%d" % world, "per_gpu_batch": B,
                       "optimizer": "momentum 0.9 (TF1)", "hip_graph": runner.graph is not None,
                       "last_loss": round(float(prog.loss.item()) / B, 4)},
        }), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
