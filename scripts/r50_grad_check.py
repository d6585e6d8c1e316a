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
from test_resnet import _cos, _ref_forward, _rel  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--arch", default="resnet50")
    ap.add_argument("--show", type=int, default=400)
    ap.add_argument("--round", action="store_true", help="oracle rounds forward activations at the bf16 storage points")
    a = ap.parse_args()
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


if __name__ == "__main__":
    main()
