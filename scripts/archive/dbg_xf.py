"""Debug: BN-on-load (xf) conv vs materialised h (round 5)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import dtfe  # noqa
from dtfe import ops

dev = torch.device("cuda", 0)
for (B, H, C, CO, K, s) in [(2, 14, 256, 256, 3, 1), (2, 14, 256, 256, 1, 1), (2, 16, 256, 256, 1, 1), (2, 14, 64, 64, 3, 1), (2, 14, 128, 128, 1, 1)]:
    pad = (K - 1) // 2
    OH = (H + 2 * pad - K) // s + 1
    g = dict(B=B, H=H, W=H, C=C, Cout=CO, OH=OH, OW=OH, KH=K, KW=K, stride=s, pad=pad)
    torch.manual_seed(1)
    x = (torch.randn(B, H, H, C, device=dev) * 1.5 + 0.3).to(torch.bfloat16)
    gamma, beta = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev) * 0.5
    st = torch.zeros(2 * C, device=dev)
    ops.bn_stats(x, st)
    h = torch.empty_like(x)
    ops.bn_apply(x, st, gamma, beta, h)
    xf = torch.empty(2 * C, device=dev)
    ops.bn_finalize(x, st, gamma, beta, xf)
    href = torch.relu(x.float() * xf[:C] + xf[C:]).to(torch.bfloat16)
    print("case", (B, H, C, CO, K, s), "h vs torch-ref mismatches:", int((h != href).sum()))
    if K == 1 and C == CO:
        w = torch.eye(C, device=dev).reshape(C, 1, 1, C).to(torch.bfloat16)
        y1 = torch.empty(B, OH, OH, CO, dtype=torch.bfloat16, device=dev)
        ops.conv_fwd(x, w, None, y1, None, g, act=ops.ACT_NONE, xf=xf)
        bad = (y1 != h)
        print("  identity conv(xf) vs h: mismatches", int(bad.sum()), "of", bad.numel())
        if bad.any():
            idx = bad.nonzero()[:8]
            print("  first bad idx", idx.tolist())
            print("  chans with bad", torch.unique(bad.nonzero()[:, 3]).tolist()[:40])
            print("  pix with bad", torch.unique(bad.reshape(-1, C).any(1).nonzero()[:, 0]).tolist()[:40])
            for b_, i_, j_, c_ in idx.tolist()[:6]:
                xv = float(x[b_, i_, j_, c_]); sc = float(xf[c_]); sh = float(xf[C + c_])
                exact = xv * sc + sh
                print("   x=%r sc=%r sh=%r exact=%r h(apply)=%r y1(xf)=%r bits h=%04x y1=%04x" % (
                    xv, sc, sh, exact, float(h[b_, i_, j_, c_]), float(y1[b_, i_, j_, c_]),
                    h[b_, i_, j_, c_].view(torch.int16).item() & 0xffff, y1[b_, i_, j_, c_].view(torch.int16).item() & 0xffff))
    w = (torch.randn(CO, K, K, C, device=dev) / (K * K * C) ** 0.5).to(torch.bfloat16)
    ya = torch.empty(B, OH, OH, CO, dtype=torch.bfloat16, device=dev)
    yb = torch.empty_like(ya)
    ops.conv_fwd(h, w, None, ya, None, g, act=ops.ACT_NONE)
    ops.conv_fwd(x, w, None, yb, None, g, act=ops.ACT_NONE, xf=xf)
    d = (ya.float() - yb.float()).abs()
    print("  conv(h) vs conv(x, xf): mismatches", int((ya != yb).sum()), "max", float(d.max()))
    if (ya != yb).any():
        print("  rows with bad:", torch.unique((ya != yb).reshape(-1, CO).any(1).nonzero()[:, 0]).tolist()[:30])
