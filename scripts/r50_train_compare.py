"""Loss trajectory of dtfe's ResNet training step (bf16 storage, HIP kernels, TF1 Momentum) next to
an fp32 autograd model started from the SAME weights and fed the SAME batches, on the GPU.  Tells a
kernel / program error (the curves part at step 1) from the training dynamics of the config
(both curves do the same thing).

    python scripts/r50_train_compare.py [--batch 256] [--steps 30] [--lr 0.1]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import torch  # noqa: E402

import dtfe  # noqa: E402,F401
from dtfe.models.resnet import ResNetModel  # noqa: E402
from dtfe.optim import Optimizer  # noqa: E402
from test_resnet import _ref_forward  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--arch", default="resnet50")
    ap.add_argument("--lr", type=float, default=0.1)
    ap.add_argument("--pool", type=int, default=512)
    ap.add_argument("--device", default="cuda")
    a = ap.parse_args()
    dev = torch.device(a.device)
    model = ResNetModel(arch=a.arch, lr=a.lr)
    B = a.batch
    prog = model.program(dev, B, seed=0)
    cfg, names, bp = model.opt_groups[0]
    gstep = torch.zeros(1, dtype=torch.int32, device=dev)
    opt = Optimizer(cfg, prog.P, var_list=names, global_step=gstep, beta_power_names=bp)
    params = {s.name: prog.P.view(s.name).detach().float().clone().reshape(s.shape).requires_grad_(True)
              for s in model.specs}
    bufs = {n: torch.zeros_like(params[n]) for n in names}
    g = torch.Generator(device=dev).manual_seed(3)
    images = torch.rand(a.pool, model.image, model.image, model.channels, device=dev, generator=g)
    labels = torch.randint(0, model.num_classes, (a.pool,), device=dev, generator=g)
    print("step  dtfe_loss  fp32_ref_loss")
    for step in range(a.steps):
        idx = torch.randint(0, a.pool, (B,), device=dev, generator=g)
        x = images[idx]
        y = torch.nn.functional.one_hot(labels[idx], model.num_classes).float()
        prog.load_batch((x, y))
        m = prog.compute_grads()
        opt.step()
        for p in params.values():
            p.grad = None
        loss, _ = _ref_forward(model, prog.P, prog.x, y, device=dev, params=params)
        with torch.no_grad():
            for n in names:
                bufs[n].mul_(0.9).add_(params[n].grad)
                params[n].sub_(a.lr * bufs[n])
        print("%4d  %9.4f  %9.4f" % (step, float(m["loss"].item()), loss.item()), flush=True)


if __name__ == "__main__":
    main()
