"""Implicit-GEMM tile variants (csrc/kernels/igemm.hip): every tile (64x64, 128x64, 128x128)
accumulates each output element over the same k-tiles in the same order with the same MFMA, so
every tile must give BITWISE the
same forward / data-gradient output (and the same fused BatchNorm partial statistics) - and the
result must match the fp32 CPU reference.  DTFE_IG_TILE forces the tile; DTFE_IG_SPLIT=1 keeps
split-K out of the comparison (split-K changes the summation order)."""
import os

import pytest
import torch

import dtfe  # noqa: F401

TILES = ["64x64", "128x64", "128x128"]

CASES = [  # (B, H, Cin, Cout, K, stride)
    (4, 14, 256, 256, 3, 1),    # 9 taps, 36 k-tiles
    (8, 28, 128, 128, 3, 2),    # strided: 4-phase data gradient
    (4, 28, 512, 128, 1, 1),    # 1x1 (N = 128)
    (3, 15, 64, 64, 3, 1),      # odd rows: partial last tile, N = 64
    (2, 14, 1024, 256, 1, 2),   # strided 1x1 projection
]


def _rel(a, b):
    return float((a.float() - b.float()).norm() / (b.float().norm() + 1e-12))


def _geom(B, H, C, CO, K, s):
    pad = (K - 1) // 2
    OH = (H + 2 * pad - K) // s + 1
    return dict(B=B, H=H, W=H, C=C, Cout=CO, OH=OH, OW=OH, KH=K, KW=K, stride=s, pad=pad)


def _run(tile, fn):
    old = {k: os.environ.get(k) for k in ("DTFE_IG_TILE", "DTFE_IG_SPLIT")}
    os.environ["DTFE_IG_TILE"] = tile
    os.environ["DTFE_IG_SPLIT"] = "1"
    try:
        out = fn()
        torch.cuda.synchronize()
        return out
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES)
def test_igemm_tiles_fwd_dgrad_bitwise(case):
    from dtfe import ops
    B, H, C, CO, K, s = case
    g = _geom(*case)
    OH = g["OH"]
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    x = torch.randn(B, H, H, C).to(torch.bfloat16)
    w = (torch.randn(CO, K, K, C) / (K * K * C) ** 0.5).to(torch.bfloat16)
    wt = w.permute(3, 1, 2, 0).contiguous()
    dy = torch.randn(B, OH, OH, CO).to(torch.bfloat16)
    base = torch.randn(B, H, H, C).to(torch.bfloat16)
    # CPU references
    y_ref = torch.empty(B, OH, OH, CO, dtype=torch.bfloat16)
    ops.conv_fwd(x, w, None, y_ref, None, g, act=ops.ACT_NONE)
    dx_ref = torch.empty(B, H, H, C, dtype=torch.bfloat16)
    ops.conv_dgrad(dy, wt, dx_ref, g)
    xd, wd, wtd, dyd, based = (t.to(dev) for t in (x, w, wt, dy, base))

    def fwd():
        y = torch.empty(B, OH, OH, CO, dtype=torch.bfloat16, device=dev)
        st = torch.zeros(2 * CO, device=dev)
        ops.conv_fwd(xd, wd, None, y, None, g, act=ops.ACT_NONE, stats=st)
        return y, st

    def dgrad():
        dx = torch.empty(B, H, H, C, dtype=torch.bfloat16, device=dev)
        ops.conv_dgrad(dyd, wtd, dx, g)
        dxa = based.clone()
        ops.conv_dgrad(dyd, wtd, dxa, g, accumulate=True)
        return dx, dxa

    res = {t: (_run(t, fwd), _run(t, dgrad)) for t in TILES if CO % int(t.split("x")[1]) == 0}
    ref_tile = "128x64"
    (y0, st0), (dx0, dxa0) = res[ref_tile]
    assert _rel(y0.cpu(), y_ref) < 2e-2
    assert _rel(dx0.cpu(), dx_ref) < 2e-2
    acc_ref = (base.float() + dx0.cpu().float())
    assert _rel(dxa0.cpu(), acc_ref) < 2e-2
    for t, ((y, st), (dx, dxa)) in res.items():
        assert torch.equal(y, y0), t
        assert torch.equal(dx, dx0), t
        assert torch.equal(dxa, dxa0), t
        # the statistics fold tiles of different heights in a different order: equal to fp32 rounding
        assert _rel(st, st0) < 1e-5, t


@pytest.mark.gpu
@pytest.mark.parametrize("tile", ["64x64", "128x64", "128x128"])
def test_igemm_tiles_bn_bwd_stats(tile):
    """The data-gradient epilogue's BN-backward statistics on every tile kernel equal a separate
    bn_bwd_stats pass over the same finished dx."""
    from dtfe import ops
    B, H, C, CO, K, s = 4, 28, 128, 256, 3, 2
    g = _geom(B, H, C, CO, K, s)
    dev = torch.device("cuda", 0)
    torch.manual_seed(1)
    OH = g["OH"]
    dy = torch.randn(B, OH, OH, CO, device=dev).to(torch.bfloat16)
    wt = (torch.randn(C, K, K, CO, device=dev) / (K * K * CO) ** 0.5).to(torch.bfloat16)
    x = torch.randn(B, H, H, C, device=dev).to(torch.bfloat16)
    mean, invstd = torch.randn(C, device=dev) * 0.1, torch.rand(C, device=dev) + 0.5
    gamma, beta = torch.randn(C, device=dev), torch.randn(C, device=dev)

    def go():
        dx = torch.empty(B, H, H, C, dtype=torch.bfloat16, device=dev)
        st = torch.zeros(2 * C, device=dev)
        ops.conv_dgrad(dy, wt, dx, g, bn_bwd=(x, None, mean, invstd, gamma, beta, st, ops.ACT_RELU))
        return dx, st

    dx, st = _run(tile, go)
    st2 = torch.zeros(2 * C, device=dev)
    ops.bn_bwd_stats(dx, None, x, mean, invstd, st2, ops.ACT_RELU, gamma=gamma, beta=beta)
    torch.cuda.synchronize()
    assert _rel(st[:C], st2[:C]) < 1e-4 and _rel(st[C:], st2[C:]) < 1e-4



W3_CASES = [  # (B, H, Cin, Cout): 3x3 / stride 1 weight gradients on the all-taps kernel
    (2, 56, 64, 64),
    (3, 28, 128, 128),
    (4, 14, 256, 64),
    (5, 7, 64, 128),
    (2, 13, 64, 64),     # W does not divide 64: partial k-tiles, ragged last row block
]


@pytest.mark.gpu
@pytest.mark.parametrize("case", W3_CASES)
@pytest.mark.parametrize("split", ["1", "0"])
def test_igemm_wgrad_all_taps_kernel(case, split):
    """igemm_wgrad3_kernel (9 taps from one staged patch) against the fp32 CPU reference and the
    per-tap kernel (DTFE_IG_W3=0); split '1' = one workgroup per tile, '0' = the automatic m-split."""
    from dtfe import ops
    B, H, C, CO = case
    g = _geom(B, H, C, CO, 3, 1)
    dev = torch.device("cuda", 0)
    torch.manual_seed(3)
    x = torch.randn(B, H, H, C).to(torch.bfloat16)
    dy = torch.randn(B, H, H, CO).to(torch.bfloat16)
    ref = torch.zeros(CO, 3, 3, C)
    ops.conv_wgrad(dy, x, ref, None, g, 0.5)
    out = {}
    for w3 in ("1", "0"):
        old = {k: os.environ.get(k) for k in ("DTFE_IG_W3", "DTFE_IG_WSPLIT")}
        os.environ["DTFE_IG_W3"], os.environ["DTFE_IG_WSPLIT"] = w3, split
        try:
            dw = torch.full((CO, 3, 3, C), 0.25, device=dev)
            ops.conv_wgrad(dy.to(dev), x.to(dev), dw, None, g, 0.5)
            torch.cuda.synchronize()
            out[w3] = dw.cpu() - 0.25
        finally:
            for k, v in old.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
    assert _rel(out["1"], ref) < 1e-2
    assert _rel(out["1"], out["0"]) < 1e-3

