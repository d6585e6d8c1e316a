"""ResNet-50 bench-shaped gradient check on the GPU: dtfe's bf16 program (the exact kernels, tile
picks, split-K / weight-gradient splits and fused BN-statistics epilogues of batch B) against an
fp32 autograd model with the same weights and batch, also on the GPU.  Prints the loss pair and
the per-variable gradient cosine / relative error, worst first.

    python scripts/r50_grad_check.py [--batch 256] [--arch resnet50]
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
from test_resnet import _cos, _ref_forward, _rel, grad_parity_table  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--arch", default="resnet50")
    ap.add_argument("--show", type=int, default=400)
    ap.add_argument("--round", action="store_true", help="oracle rounds forward activations at the bf16 storage points")
    ap.add_argument("--amp", action="store_true", help="per-variable cos of dtfe AND of stock autocast-bf16 vs fp32")
    a = ap.parse_args()
    if a.amp:
        return amp_table(a)
    model = ResNetModel(arch=a.arch)
    torch.manual_seed(0)
    B, dev = a.batch, torch.device("cuda", 0)
    prog = model.program(dev, B, seed=1)
    x = torch.rand(B, model.image, model.image, model.channels, device=dev)
    y = torch.nn.functional.one_hot(torch.randint(0, model.num_classes, (B,), device=dev), model.num_classes).float()
    prog.load_batch((x, y))
    m = prog.compute_grads()
    torch.cuda.synchronize()
    loss, params = _ref_forward(model, prog.P, prog.x, y, device=dev, round_act=a.round)
    print("loss dtfe %.5f ref %.5f" % (float(m["loss"].item()), loss.item()))
    rows = []
    names = [s.name for s in model.specs if not s.name.endswith(("moving_mean", "moving_variance"))]
    for n in names:
        g = prog.P.gview(n).detach().float()
        r = params[n].grad
        rows.append((_cos(g, r), _rel(g, r), float(g.norm()), float(r.norm()), n))
    for c, e, gn, rn, n in rows[: a.show]:  # backward order: head first
        print("cos %.4f rel %.4f |g| %.4e |ref| %.4e  %s" % (c, e, gn, rn, n))
    rows.sort()
    print("min cos %.4f, median cos %.4f over %d variables" % (rows[0][0], rows[len(rows) // 2][0], len(rows)))


def amp_table(a):
    model = ResNetModel(arch=a.arch)
    torch.manual_seed(0)
    B, dev = a.batch, torch.device("cuda", 0)
    prog = model.program(dev, B, seed=1)
    x = torch.rand(B, model.image, model.image, model.channels, device=dev)
    y = torch.nn.functional.one_hot(torch.randint(0, model.num_classes, (B,), device=dev), model.num_classes).float()
    rows = grad_parity_table(model, prog, x, y, dev)
    print("# B=%d %s: gradient cosine vs the fp32 autograd model (same weights, same batch); backward order" %
          (B, a.arch))
    print("%-44s %9s %9s %8s" % ("variable", "cos dtfe", "cos amp", "delta"))
    for n, cd, ca in rows:
        print("%-44s %9.4f %9.4f %+8.4f" % (n, cd, ca, cd - ca))
    convs = [r for r in rows if r[0].endswith("/kernel") and "conv2d" in r[0]]
    print("conv kernels: mean cos dtfe %.4f amp %.4f; min dtfe %.4f amp %.4f; dtfe worse than amp-0.05 on %d of %d" % (
        sum(r[1] for r in convs) / len(convs), sum(r[2] for r in convs) / len(convs), min(r[1] for r in convs),
        min(r[2] for r in convs), sum(r[1] < r[2] - 0.05 for r in convs), len(convs)))


if __name__ == "__main__":
    main()
