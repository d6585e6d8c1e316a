import os, sys
sys.path.insert(0, os.getcwd())
import torch
import dtfe
from dtfe import ops
for (B, H, C, Cout, k) in [(16, 28, 128, 256, 3), (3, 14, 64, 128, 3)]:
    torch.manual_seed(3)
    x = torch.randn(B, H, H, C, device="cuda").to(torch.bfloat16)
    w = (torch.randn(Cout, k, k, C, device="cuda") * 0.05).to(torch.bfloat16)
    g = dict(B=B, H=H, W=H, C=C, Cout=Cout, OH=H, OW=H, KH=k, KW=k, stride=1, pad=(k - 1) // 2)
    y1 = torch.empty(B, H, H, Cout, device="cuda", dtype=torch.bfloat16)
    s1 = torch.zeros(2 * Cout, device="cuda")
    ops.conv_fwd(x, w, None, y1, None, g, act=ops.ACT_NONE, stats=s1)
    torch.cuda.synchronize()
    s2 = torch.zeros(2 * Cout, device="cuda")
    ops.bn_stats(y1, s2)
    torch.cuda.synchronize()
    print(B, H, C, Cout, k, "fused", s1[:4].tolist(), s1[Cout:Cout + 4].tolist(), "sep", s2[:4].tolist(), s2[Cout:Cout+4].tolist())
