#!/usr/bin/env python
"""Row (a) of BASELINE.md: the same MNIST CNN in *stock* PyTorch-ROCm
(nn.Conv2d/Linear via MIOpen + hipBLASLt, bf16 autocast, torch.optim.Adam,
DistributedDataParallel over RCCL), timed with the same harness as bench.py.
--graph: the honest 1-GPU bar - the whole step (sampling, fwd, bwd, fused Adam)
captured into one HIP graph, no per-op launch overhead.

    python bench/stock_torch_cnn.py --steps 100 --warmup 20 --batch_size 1024 [--write]
    torchrun --nproc-per-node N bench/stock_torch_cnn.py ...

--write records the result in bench/stock_baseline.json (key "<N>x<batch>"),
which bench.py divides by for vs_baseline.
"""
import argparse
import json
import os
import time

import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F


class Net(nn.Module):
    def __init__(self):
        super().__init__()
        self.c1 = nn.Conv2d(1, 32, 5, padding=2)
        self.c2 = nn.Conv2d(32, 64, 5, padding=2)
        self.f1 = nn.Linear(3136, 1024)
        self.f2 = nn.Linear(1024, 10)
        self.drop = nn.Dropout(0.25)

    def forward(self, x):
        x = F.max_pool2d(F.relu(self.c1(x)), 2)
        x = F.max_pool2d(F.relu(self.c2(x)), 2)
        x = self.drop(F.relu(self.f1(x.flatten(1))))
        return self.f2(x)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch_size", type=int, default=1024)
    ap.add_argument("--write", action="store_true")
    ap.add_argument("--dtype", choices=["bf16", "fp32"], default="bf16",
                    help="bf16 autocast (the headline row) or plain fp32 (the reference's precision)")
    ap.add_argument("--graph", action="store_true", help="capture the whole step (fwd, bwd, fused optimizer) in one "
                    "CUDA/HIP graph (1 GPU); implies --fused")
    ap.add_argument("--fused", action="store_true", help="torch.optim fused=True optimizer kernels")
    a = ap.parse_args()
    a.fused = a.fused or a.graph
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    lr_ = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(lr_)
    dev = torch.device("cuda", lr_)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    net = Net().to(dev).to(memory_format=torch.channels_last)
    model = nn.parallel.DistributedDataParallel(net, device_ids=[lr_]) if world > 1 else net
    opt = torch.optim.Adam(model.parameters(), lr=1e-3, fused=True, capturable=a.graph) if a.fused \
        else torch.optim.Adam(model.parameters(), lr=1e-3)
    g = torch.Generator(device=dev).manual_seed(0)
    data = torch.randint(0, 256, (60000, 1, 28, 28), device=dev, dtype=torch.uint8, generator=g)
    labels = torch.randint(0, 10, (60000,), device=dev, generator=g)

    n_pool_, B_ = 60000, a.batch_size

    def xform(idx):
        return (data[idx].float() / 255).contiguous(memory_format=torch.channels_last)

    def step():
        idx = torch.randint(0, 60000, (a.batch_size,), device=dev, generator=g)
        x = (data[idx].float() / 255).contiguous(memory_format=torch.channels_last)
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=a.dtype == "bf16"):
            loss = F.cross_entropy(model(x), labels[idx])
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()
        return loss

    runner = step
    if a.graph:
        assert world == 1, "--graph is the 1-GPU stock row (DDP steps stay eager)"

        def gstep():  # the captured step: backward ASSIGNS fresh grads (set to None before capture)
            idx = torch.randint(0, n_pool_, (B_,), device=dev)
            x = xform(idx)
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=a.dtype == "bf16"):
                loss = F.cross_entropy(model(x), labels[idx])
            loss.backward()
            opt.step()
            return loss

        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(3):
                opt.zero_grad(set_to_none=True)
                gstep()
        torch.cuda.current_stream().wait_stream(s)
        G = torch.cuda.CUDAGraph()
        opt.zero_grad(set_to_none=True)
        with torch.cuda.graph(G):
            gstep()
        runner = G.replay
    for _ in range(a.warmup):
        runner()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        runner()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = t.item()
    v = a.batch_size * world * a.steps / el
    if rank == 0:
        print(json.dumps({"stock_torch_images_per_sec": round(v, 1), "dtype": a.dtype, "n_gpus": world, "batch_size": a.batch_size,
                          "ms_per_step": round(el / a.steps * 1000, 3), "graph": a.graph, "fused_optimizer": a.fused}),
              flush=True)
        if a.write:
            p = os.path.join(os.path.dirname(os.path.abspath(__file__)), "stock_baseline.json")
            tab = {}
            if os.path.exists(p):
                tab = json.load(open(p))
            tab[f"{world}x{a.batch_size}" + ("_graph_fused" if a.graph else "_fused" if a.fused else "")] = round(v, 1)
            json.dump(tab, open(p, "w"), indent=1, sort_keys=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
