"""Localise imgwgrad mismatches: vary batch (images per block), pooled dy, geometry."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dtfe  # noqa: E402,F401
import dtfe.ops as ops  # noqa: E402


def run(B, SH, CS, N, K, s, pad, pooled, seed=0):
    OH = (SH + 2 * pad - K) // s + 1
    torch.manual_seed(seed)
    x = torch.randn(B, SH, SH, CS).cuda().to(torch.bfloat16)
    kw = dict(B=B, SH=SH, SW=SH, CS=CS, OH=OH, OW=OH, N=N, KH=K, KW=K, stride=s, pad=pad)
    dw = torch.zeros(N, K, K, CS, device="cuda")
    dwr = torch.zeros(N, K, K, CS)
    if pooled:
        dp = torch.randn(B, OH // 2, OH // 2, N).cuda().to(torch.bfloat16)
        am = torch.randint(0, 4, dp.shape, dtype=torch.uint8).cuda()
        ops.imgwgrad(x, dw, None, dy_pooled=dp, dy_argmax=am, **kw)
        ops.imgwgrad(x.cpu(), dwr, None, dy_pooled=dp.cpu(), dy_argmax=am.cpu(), **kw)
    else:
        dy = torch.randn(B, OH, OH, N).cuda().to(torch.bfloat16)
        ops.imgwgrad(x, dw, None, dy=dy, **kw)
        ops.imgwgrad(x.cpu(), dwr, None, dy=dy.cpu(), **kw)
    d = (dw.cpu() - dwr).abs()
    rel = (d.max() / dwr.abs().max()).item()
    # where are the errors: per output channel / per tap / per cin
    bad_n = (d.amax(dim=(1, 2, 3)) > 0.05 * dwr.abs().max()).nonzero().flatten().tolist()
    bad_tap = (d.amax(dim=(0, 3)) > 0.05 * dwr.abs().max()).nonzero().tolist()
    bad_c = (d.amax(dim=(0, 1, 2)) > 0.05 * dwr.abs().max()).nonzero().flatten().tolist()
    print(f"B={B} SH={SH} CS={CS} N={N} K={K} s={s} pooled={pooled}: rel={rel:.4f} bad_n={bad_n[:8]}"
          f" bad_tap={bad_tap[:6]} bad_c={bad_c[:8]}", flush=True)


for cfg in [(1, 14, 32, 64, 5, 1, 2, False), (1, 14, 32, 64, 5, 1, 2, True), (5, 14, 32, 64, 5, 1, 2, False),
            (5, 14, 32, 64, 5, 1, 2, True), (3, 32, 16, 16, 3, 1, 1, False), (1, 8, 64, 64, 3, 1, 1, False),
            (1, 14, 32, 16, 5, 1, 2, False), (1, 14, 32, 32, 5, 1, 2, False), (1, 8, 8, 16, 3, 1, 1, False),
            (1, 8, 16, 16, 1, 1, 0, False)]:
    run(*cfg)
