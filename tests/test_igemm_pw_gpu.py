"""The persistent pipelined implicit-GEMM kernel (csrc/kernels/igemm_pw.hip) vs fp32 references and
vs the per-tile implicit-GEMM kernel (DTFE_PW=off).

Covers: 1x1 and 3x3 forward at stride 1 / 2 with the fused BatchNorm statistics, stride-1 data
gradients (1x1, 3x3 with flipped taps), the stride-2 1x1 data gradient that accumulates onto the
shortcut's share, M not a multiple of the tile, every tile / ring configuration (DTFE_PW cfg=) and
small grids that make every workgroup stream several tiles (the k-tile stream crossing tile
boundaries, DTFE_PW grid=).  mintiles=1 keeps these small shapes on the persistent path."""
import pytest
import torch
import torch.nn.functional as F

import dtfe  # noqa: F401
from dtfe import ops

pytestmark = pytest.mark.gpu
DEV = "cuda"

CASES = [  # B, H, C, Cout, stride, k
    (2, 9, 64, 64, 1, 1),       # M = 162: partial last tile, 1 k-tile
    (3, 14, 256, 64, 1, 1),     # reduce, 4 k-tiles, N = 64 (128x64 tiles)
    (2, 14, 64, 256, 1, 1),     # expand, N = 256
    (2, 7, 512, 128, 1, 1),     # 8 k-tiles
    (2, 14, 256, 512, 2, 1),    # strided projection (7x7 output)
    (1, 28, 128, 512, 1, 1),    # 784 rows
    (2, 14, 64, 64, 1, 3),      # 3x3: 9 taps, border taps read the zero page
    (2, 15, 128, 128, 2, 3),    # strided 3x3 (v1.5), odd image
    (2, 7, 256, 128, 1, 3),     # 3x3, 4 k-tiles per tap
]


def _stats_ref(y):
    """(sum (y - y0), sum (y - y0)^2) per channel, y0 = row 0 - the shifted form of dtfe.ops.bn_stats."""
    yf = y.double().reshape(-1, y.shape[-1])
    d = yf - yf[0:1]
    return torch.stack([d.sum(0), (d * d).sum(0)])


def _pw(monkeypatch, **kw):
    """DTFE_PW=all,<k>=<v>... (every one-phase launch on the persistent kernel, small shapes too)"""
    monkeypatch.setenv("DTFE_PW", ",".join(["all", "mintiles=1"] + ["%s=%s" % kv for kv in kw.items()]))


@pytest.fixture(params=[None, "0", "1", "2", "3"])
def cfg(request, monkeypatch):
    _pw(monkeypatch, **({} if request.param is None else {"cfg": request.param}))
    return request.param


@pytest.mark.parametrize("grid", [None, "5"])
@pytest.mark.parametrize("case", CASES)
def test_pw_fwd_with_bn_stats(case, grid, cfg, monkeypatch):
    B, H, C, Cout, s, k = case
    if grid:
        _pw(monkeypatch, grid=grid, **({} if cfg is None else {"cfg": cfg}))
    pad = (k - 1) // 2
    OH = (H + 2 * pad - k) // s + 1
    g = dict(B=B, H=H, W=H, C=C, Cout=Cout, OH=OH, OW=OH, KH=k, KW=k, stride=s, pad=pad)
    torch.manual_seed(1)
    x = torch.randn(B, H, H, C).to(torch.bfloat16)
    w = (torch.randn(Cout, k, k, C) / (k * C ** 0.5)).to(torch.bfloat16)
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), stride=s,
                   padding=pad).permute(0, 2, 3, 1)
    y = torch.full((B, OH, OH, Cout), float("nan"), device=DEV, dtype=torch.bfloat16)
    st = torch.zeros(2, Cout, device=DEV)
    ops.conv_fwd(x.to(DEV), w.to(DEV), None, y, None, g, act=ops.ACT_NONE, stats=st)
    torch.cuda.synchronize()
    assert torch.isfinite(y.float()).all()
    err = (y.float().cpu() - ref).abs().max().item()
    assert err <= 1e-2 * ref.abs().max().item(), err
    sr = _stats_ref(y.cpu())
    assert torch.allclose(st.double().cpu(), sr, rtol=1e-4, atol=1e-3 * B * OH * OH), (st.cpu(), sr)
    # the per-tile implicit-GEMM kernel computes the same products: identical output
    monkeypatch.setenv("DTFE_PW", "off")
    y2 = torch.empty_like(y)
    st2 = torch.zeros_like(st)
    ops.conv_fwd(x.to(DEV), w.to(DEV), None, y2, None, g, act=ops.ACT_NONE, stats=st2)
    torch.cuda.synchronize()
    assert (y.float() - y2.float()).abs().max().item() <= 1e-2 * ref.abs().max().item()


@pytest.mark.parametrize("grid", [None, "3"])
@pytest.mark.parametrize("case", CASES)
def test_pw_dgrad(case, grid, cfg, monkeypatch):
    B, H, C, Cout, s, k = case
    if grid:
        _pw(monkeypatch, grid=grid, **({} if cfg is None else {"cfg": cfg}))
    pad = (k - 1) // 2
    OH = (H + 2 * pad - k) // s + 1
    g = dict(B=B, H=H, W=H, C=C, Cout=Cout, OH=OH, OW=OH, KH=k, KW=k, stride=s, pad=pad)
    torch.manual_seed(2)
    w = (torch.randn(Cout, k, k, C) / (k * Cout ** 0.5)).to(torch.bfloat16)
    dy = torch.randn(B, OH, OH, Cout).to(torch.bfloat16)
    ref = torch.nn.grad.conv2d_input((B, C, H, H), w.float().permute(0, 3, 1, 2), dy.float().permute(0, 3, 1, 2),
                                     stride=s, padding=pad).permute(0, 2, 3, 1)
    wt = w.permute(3, 1, 2, 0).contiguous().to(DEV)
    base = torch.randn(B, H, H, C).to(torch.bfloat16)
    # the strided 1x1 data gradient always accumulates (projection shortcut); a strided 3x3 data
    # gradient (four parity phases) stays on the per-tile kernel - test it accumulating too
    accumulate = s == 2
    dx = base.to(DEV) if accumulate else torch.full((B, H, H, C), float("nan"), device=DEV, dtype=torch.bfloat16)
    ops.conv_dgrad(dy.to(DEV), wt, dx, g, accumulate=accumulate)
    torch.cuda.synchronize()
    want = ref + (base.float() if accumulate else 0)
    err = (dx.float().cpu() - want).abs().max().item()
    assert err <= 2e-2 * want.abs().max().item(), err
    if accumulate and k == 1:  # phases no tap reaches keep the shortcut's share bit for bit
        m = torch.ones(H, H, dtype=torch.bool)
        m[::2, ::2] = False
        assert torch.equal(dx.cpu()[:, m], base[:, m])


def test_pw_large_m_many_tiles_per_workgroup(monkeypatch):
    """ResNet-50 stage-1 expand at batch 16 (M = 50176): every workgroup streams ~100 tiles."""
    _pw(monkeypatch)
    B, H, C, Cout = 16, 56, 64, 256
    g = dict(B=B, H=H, W=H, C=C, Cout=Cout, OH=H, OW=H, KH=1, KW=1, stride=1, pad=0)
    torch.manual_seed(3)
    x = torch.randn(B, H, H, C, device=DEV).to(torch.bfloat16)
    w = (torch.randn(Cout, 1, 1, C, device=DEV) / 8).to(torch.bfloat16)
    y = torch.empty(B, H, H, Cout, device=DEV, dtype=torch.bfloat16)
    st = torch.zeros(2, Cout, device=DEV)
    ops.conv_fwd(x, w, None, y, None, g, act=ops.ACT_NONE, stats=st)
    ref = (x.float().reshape(-1, C) @ w.float().reshape(Cout, C).t()).reshape(y.shape)
    torch.cuda.synchronize()
    assert (y.float() - ref).abs().max().item() <= 1e-2 * ref.abs().max().item()
    sr = _stats_ref(y)
    assert torch.allclose(st.double(), sr, rtol=1e-4, atol=1.0)
