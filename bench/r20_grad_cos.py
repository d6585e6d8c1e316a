#!/usr/bin/env python
"""ResNet-20 B=256 default schedule vs fp32 autograd (tests/test_resnet.py's bench-shaped oracle):
per-variable relative error / cosine, with and without the conv-fused output BN statistics
(models/resnet.py _OUT_STATS).   python bench/r20_grad_cos.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import dtfe  # noqa: E402,F401
import dtfe.models.resnet as R  # noqa: E402
from test_resnet import _cos, _ref_forward, _rel  # noqa: E402

B = 256
res = {}
for fused in (False, True):
    R._OUT_STATS = fused
    model = R.ResNetModel(arch="resnet20")
    torch.manual_seed(0)
    prog = model.program("cuda", B, seed=1)
    x = torch.rand(B, 32, 32, 3, device="cuda")
    y = F.one_hot(torch.randint(0, 10, (B,), device="cuda"), 10).float()
    prog.load_batch((x, y))
    m = prog.compute_grads()
    torch.cuda.synchronize()
    loss, ref = _ref_forward(model, prog.P, prog.x, y, device="cuda", round_act=True)
    names = [s.name for s in model.specs if not s.name.endswith(("moving_mean", "moving_variance"))]
    res[fused] = {n: (_rel(prog.P.gview(n).float(), ref[n].grad.float()), _cos(prog.P.gview(n).float(), ref[n].grad.float()))
                  for n in names}
    print("fused=%d loss %.6f ref %.6f" % (fused, float(m["loss"]), float(loss)))
print("%-44s %10s %8s %10s %8s" % ("variable", "rel", "cos", "rel(fused)", "cos"))
for n in res[False]:
    a, b = res[False][n], res[True][n]
    print("%-44s %10.4f %8.4f %10.4f %8.4f" % (n, a[0], a[1], b[0], b[1]))
