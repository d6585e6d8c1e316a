#!/usr/bin/env python
"""Stock PyTorch-ROCm rows of BASELINE.md for the ResNet configurations.

This is the same ResNet-20 (CIFAR-10, option-A shortcuts) and ResNet-50
(ImageNet shape, projection shortcuts) that ``dtfe.models.resnet`` builds, here
written with nn.Conv2d / nn.BatchNorm2d (MIOpen), channels_last, bf16 autocast,
SGD with momentum 0.9, and DistributedDataParallel over RCCL. It is timed with
the same harness as bench.py: device-resident uint8 images, device-side
sampling, and K timed steps bracketed by synchronize + barrier.

    python bench/stock_torch_resnet.py --arch resnet20 --batch_size 256 [--write]
    torchrun --nproc-per-node N bench/stock_torch_resnet.py --arch resnet50 ...

--write records images/sec in bench/stock_baseline.json under the key
"<arch>_<N>x<batch>".
"""
import argparse
import json
import os
import time

import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F


class Basic(nn.Module):
    def __init__(self, cin, cout, stride):
        super().__init__()
        self.c1 = nn.Conv2d(cin, cout, 3, stride, 1, bias=False)
        self.b1 = nn.BatchNorm2d(cout, eps=1e-3, momentum=0.01)
        self.c2 = nn.Conv2d(cout, cout, 3, 1, 1, bias=False)
        self.b2 = nn.BatchNorm2d(cout, eps=1e-3, momentum=0.01)
        self.stride, self.pad = stride, cout - cin

    def forward(self, x):
        y = F.relu(self.b1(self.c1(x)))
        y = self.b2(self.c2(y))
        s = x[:, :, ::self.stride, ::self.stride] if self.stride > 1 else x
        if self.pad:
            s = F.pad(s, (0, 0, 0, 0, 0, self.pad))
        return F.relu(y + s)


class Bottleneck(nn.Module):
    def __init__(self, cin, mid, stride):
        super().__init__()
        cout = 4 * mid
        self.c1 = nn.Conv2d(cin, mid, 1, bias=False)
        self.b1 = nn.BatchNorm2d(mid, eps=1e-3, momentum=0.01)
        self.c2 = nn.Conv2d(mid, mid, 3, stride, 1, bias=False)
        self.b2 = nn.BatchNorm2d(mid, eps=1e-3, momentum=0.01)
        self.c3 = nn.Conv2d(mid, cout, 1, bias=False)
        self.b3 = nn.BatchNorm2d(cout, eps=1e-3, momentum=0.01)
        self.proj = None
        if stride != 1 or cin != cout:
            self.proj = nn.Sequential(nn.Conv2d(cin, cout, 1, stride, bias=False),
                                      nn.BatchNorm2d(cout, eps=1e-3, momentum=0.01))

    def forward(self, x):
        y = F.relu(self.b1(self.c1(x)))
        y = F.relu(self.b2(self.c2(y)))
        y = self.b3(self.c3(y))
        return F.relu(y + (self.proj(x) if self.proj is not None else x))


def resnet20():
    layers = [nn.Conv2d(3, 16, 3, 1, 1, bias=False), nn.BatchNorm2d(16, eps=1e-3, momentum=0.01), nn.ReLU()]
    cin = 16
    for stage, c in enumerate((16, 32, 64)):
        for i in range(3):
            layers.append(Basic(cin, c, 2 if (stage and i == 0) else 1))
            cin = c
    layers += [nn.AdaptiveAvgPool2d(1), nn.Flatten(), nn.Linear(64, 10)]
    return nn.Sequential(*layers), (3, 32, 32), 10


def resnet50():
    layers = [nn.Conv2d(3, 64, 7, 2, 3, bias=False), nn.BatchNorm2d(64, eps=1e-3, momentum=0.01), nn.ReLU(),
              nn.MaxPool2d(3, 2, 1)]
    cin = 64
    for stage, (mid, n) in enumerate(((64, 3), (128, 4), (256, 6), (512, 3))):
        for i in range(n):
            layers.append(Bottleneck(cin, mid, 2 if (stage and i == 0) else 1))
            cin = 4 * mid
    layers += [nn.AdaptiveAvgPool2d(1), nn.Flatten(), nn.Linear(2048, 1000)]
    return nn.Sequential(*layers), (3, 224, 224), 1000


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", choices=["resnet20", "resnet50"], default="resnet20")
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch_size", type=int, default=None)
    ap.add_argument("--write", action="store_true")
    ap.add_argument("--graph", action="store_true", help="capture the whole step (fwd, bwd, fused optimizer) in one "
                    "CUDA/HIP graph (1 GPU); implies --fused")
    ap.add_argument("--fused", action="store_true", help="torch.optim fused=True optimizer kernels")
    a = ap.parse_args()
    a.fused = a.fused or a.graph
    B = a.batch_size or (256 if a.arch == "resnet20" else 64)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    lr_ = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(lr_)
    dev = torch.device("cuda", lr_)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    net, (C, H, W), ncls = resnet20() if a.arch == "resnet20" else resnet50()
    net = net.to(dev).to(memory_format=torch.channels_last)
    model = nn.parallel.DistributedDataParallel(net, device_ids=[lr_]) if world > 1 else net
    opt = torch.optim.SGD(model.parameters(), lr=0.1, momentum=0.9, fused=True) if a.fused \
        else torch.optim.SGD(model.parameters(), lr=0.1, momentum=0.9)
    g = torch.Generator(device=dev).manual_seed(rank)
    n_pool = 4096 if a.arch == "resnet20" else 512
    data = torch.randint(0, 256, (n_pool, H, W, C), device=dev, dtype=torch.uint8, generator=g)
    labels = torch.randint(0, ncls, (n_pool,), device=dev, generator=g)

    n_pool_, B_ = n_pool, B

    def xform(idx):
        return (data[idx].float() / 255).permute(0, 3, 1, 2)

    def step():
        idx = torch.randint(0, n_pool, (B,), device=dev, generator=g)
        x = (data[idx].float() / 255).permute(0, 3, 1, 2)  # NHWC storage == channels_last NCHW view
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = F.cross_entropy(model(x), labels[idx])
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()
        return loss

    out = {}

    def runner_eager():
        out["loss"] = step()

    runner = runner_eager
    if a.graph:
        assert world == 1, "--graph is the 1-GPU stock row (DDP steps stay eager)"

        def gstep():  # the captured step: backward ASSIGNS fresh grads (set to None before capture)
            idx = torch.randint(0, n_pool_, (B_,), device=dev)
            x = xform(idx)
            with torch.autocast("cuda", dtype=torch.bfloat16):
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
            out["loss"] = gstep()
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
    v = B * world * a.steps / el
    if rank == 0:
        print(json.dumps({"arch": a.arch, "stock_torch_images_per_sec": round(v, 1), "n_gpus": world,
                          "batch_size": B, "ms_per_step": round(el / a.steps * 1000, 3), "graph": a.graph,
                          "fused_optimizer": a.fused, "last_loss": round(float(out["loss"]), 4)}), flush=True)
        if a.write:
            p = os.path.join(os.path.dirname(os.path.abspath(__file__)), "stock_baseline.json")
            tab = json.load(open(p)) if os.path.exists(p) else {}
            tab[f"{a.arch}_{world}x{B}" + ("_graph_fused" if a.graph else "_fused" if a.fused else "")] = round(v, 1)
            json.dump(tab, open(p, "w"), indent=1, sort_keys=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
