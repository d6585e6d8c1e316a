"""Layer-by-layer forward comparison of the ResNet program on the GPU kernels vs the CPU
reference path (same weights, same bf16 storage points): where do activations diverge?"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dtfe  # noqa: E402,F401
from dtfe.models.resnet import ResNetModel  # noqa: E402

arch = sys.argv[1] if len(sys.argv) > 1 else "resnet50"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 2
model = ResNetModel(arch=arch)
torch.manual_seed(0)
x = torch.rand(B, model.image, model.image, 3)
y = torch.nn.functional.one_hot(torch.randint(0, model.num_classes, (B,)), model.num_classes).float()
acts = {}
for dev in ("cpu", "cuda"):
    p = model.program(dev, B, seed=1)
    p.load_batch((x.to(dev), y.to(dev)))
    p.P.grad.zero_(); p.arena.buf.zero_(); p.loss.zero_(); p.correct.zero_()
    p.forward()
    L = p.L
    a = [("stem_conv", L["stem"].y)]
    if "pool_hw" in L:  # (BN + ReLU + pool are one pass on the GPU: the stem BN map is not stored)
        a.append(("pool", p.pool))
    else:
        a.append(("stem_bn", L["stem_bn"].y))
    for i, b in enumerate(L["blocks"]):
        a.append(("block%d.conv1" % i, b.conv1.y))
        a.append(("block%d.out" % i, b.bn3.y if hasattr(b, "bn3") else b.bn2.y))
    a.append(("feat", p.feat))
    a.append(("logits", p.logits))
    acts[dev] = [(n, t.float().cpu()) for n, t in a]
    print(dev, "loss", float(p.loss.item()) / B)
for (n, c), (_, g) in zip(acts["cpu"], acts["cuda"]):
    print("%-16s rel %.4f   max|cpu| %.3f" % (n, ((g - c).norm() / (c.norm() + 1e-12)).item(), c.abs().max().item()))
