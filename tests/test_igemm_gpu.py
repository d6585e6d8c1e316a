"""DMA-staged implicit-GEMM convolution (csrc/kernels/igemm.hip) vs fp32 PyTorch references.

Covers every ResNet-50 conv kind (1x1 / 3x3, stride 1 / 2, projection), an odd
image size (unequal stride-2 phase grids), every tile shape (DTFE_IG_TILE) and
the split-K forward / split-M weight-gradient reductions.
"""
import os

import pytest
import torch
import torch.nn.functional as F

import dtfe  # noqa: F401
from dtfe import ops

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _geom(B, H, C, Cout, k, s):
    pad = (k - 1) // 2
    OH = (H + 2 * pad - k) // s + 1
    return dict(B=B, H=H, W=H, C=C, Cout=Cout, OH=OH, OW=OH, KH=k, KW=k, stride=s, pad=pad)


def _rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return ((a - b).abs().max() / (b.abs().max() + 1e-6)).item()


CASES = [
    (4, 14, 64, 256, 1, 1),     # bottleneck expand
    (4, 14, 256, 64, 1, 1),     # bottleneck reduce
    (2, 14, 64, 64, 3, 1),      # 3x3
    (2, 14, 128, 128, 3, 2),    # strided 3x3 (v1.5)
    (2, 14, 256, 512, 1, 2),    # strided projection
    (2, 7, 64, 128, 3, 2),      # odd image: phase grids 4x4 / 4x3 / 3x4 / 3x3
    (8, 7, 512, 512, 3, 1),     # stage-4 3x3: few tiles -> split-K forward
]


@pytest.fixture(params=["auto", "128x128", "128x64", "64x128", "64x64"])
def tile(request, monkeypatch):
    if request.param != "auto":
        monkeypatch.setenv("DTFE_IG_TILE", request.param)
    return request.param


@pytest.mark.parametrize("case", CASES)
def test_igemm_fwd_dgrad_wgrad(case, tile):
    B, H, C, Cout, k, s = case
    if tile != "auto" and int(tile.split("x")[1]) > min(C, Cout):
        pytest.skip("tile wider than the channel count")
    g = _geom(B, H, C, Cout, k, s)
    torch.manual_seed(1)
    x = torch.randn(B, H, H, C).to(torch.bfloat16)
    w = (torch.randn(Cout, k, k, C) / (k * (C ** 0.5))).to(torch.bfloat16)
    dy = torch.randn(B, g["OH"], g["OW"], Cout).to(torch.bfloat16)
    xn, wn, dyn = x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), dy.float().permute(0, 3, 1, 2)
    ref_y = F.conv2d(xn, wn, stride=s, padding=g["pad"]).permute(0, 2, 3, 1)
    ref_dx = torch.nn.grad.conv2d_input(xn.shape, wn, dyn, stride=s, padding=g["pad"]).permute(0, 2, 3, 1)
    ref_dw = torch.nn.grad.conv2d_weight(xn, wn.shape, dyn, stride=s, padding=g["pad"]).permute(0, 2, 3, 1)

    xd, wd, dyd = x.to(DEV), w.to(DEV), dy.to(DEV)
    wt = w.permute(3, 1, 2, 0).contiguous().to(DEV)  # [Cin][KH][KW][Cout]
    y = torch.full((B, g["OH"], g["OW"], Cout), float("nan"), device=DEV, dtype=torch.bfloat16)
    ops.conv_fwd(xd, wd, None, y, None, g, act=ops.ACT_NONE)
    dx = torch.full((B, H, H, C), float("nan"), device=DEV, dtype=torch.bfloat16)
    ops.conv_dgrad(dyd, wt, dx, g)
    dw = torch.full((Cout, k, k, C), 0.5, device=DEV)  # wgrad accumulates (+=)
    ops.conv_wgrad(dyd, xd, dw, None, g, 1.0)
    torch.cuda.synchronize()
    assert torch.isfinite(y.float()).all() and torch.isfinite(dx.float()).all()
    assert _rel(y, ref_y) < 1e-2
    assert _rel(dx, ref_dx) < 1e-2
    assert _rel(dw - 0.5, ref_dw) < 1e-3


@pytest.mark.parametrize("case", CASES)
def test_igemm_wgrad_per_tap(case, monkeypatch):
    """The per-tap weight-gradient kernel (4-stage ring of 32-pixel k-tiles) against fp32."""
    monkeypatch.setenv("DTFE_IG_W3", "0")   # the per-tap kernel for the 3x3 shapes too
    B, H, C, Cout, k, s = case
    g = _geom(B, H, C, Cout, k, s)
    torch.manual_seed(4)
    x = torch.randn(B, H, H, C).to(torch.bfloat16)
    dy = torch.randn(B, g["OH"], g["OW"], Cout).to(torch.bfloat16)
    ref = torch.nn.grad.conv2d_weight(x.float().permute(0, 3, 1, 2), (Cout, C, k, k), dy.float().permute(0, 3, 1, 2),
                                      stride=s, padding=g["pad"]).permute(0, 2, 3, 1)
    dw = torch.zeros(Cout, k, k, C, device=DEV)
    ops.conv_wgrad(dy.to(DEV), x.to(DEV), dw, None, g, 1.0)
    torch.cuda.synchronize()
    assert _rel(dw, ref) < 1e-3


def test_igemm_wgrad_scale_and_splits(monkeypatch):
    g = _geom(16, 14, 64, 64, 3, 1)
    torch.manual_seed(2)
    x = torch.randn(16, 14, 14, 64).to(torch.bfloat16)
    dy = torch.randn(16, 14, 14, 64).to(torch.bfloat16)
    ref = torch.nn.grad.conv2d_weight(x.float().permute(0, 3, 1, 2), (64, 64, 3, 3), dy.float().permute(0, 3, 1, 2),
                                      padding=1).permute(0, 2, 3, 1)
    outs = []
    for sp in ("1", "3", "0"):
        monkeypatch.setenv("DTFE_IG_WSPLIT", sp)
        dw = torch.zeros(64, 3, 3, 64, device=DEV)
        ops.conv_wgrad(dy.to(DEV), x.to(DEV), dw, None, g, 0.25)
        outs.append(dw.cpu())
    for o in outs:
        assert _rel(o, 0.25 * ref) < 1e-3


@pytest.mark.parametrize("B,H,C,Cout", [(4, 14, 256, 64), (2, 7, 512, 128), (3, 9, 64, 64)])
def test_igemm_dgrad_masked_accumulation_source(B, H, C, Cout):
    """conv_dgrad(accumulate=True, acc_src=(src, bits)): dx = dgrad + src * bit, dx's old contents
    never read - equal (bit for bit) to accumulating onto a dx pre-filled with the masked src."""
    g = _geom(B, H, C, Cout, 1, 1)
    torch.manual_seed(4)
    dy = torch.randn(B, H, H, Cout, device=DEV).to(torch.bfloat16)
    wt = (torch.randn(C, 1, 1, Cout, device=DEV) / Cout ** 0.5).to(torch.bfloat16)
    src = torch.randn(B, H, H, C, device=DEV).to(torch.bfloat16)
    y = torch.relu(torch.randn(B, H, H, C, device=DEV)).to(torch.bfloat16)
    bits = ops.relu_bits(y)
    dx = torch.full((B, H, H, C), float("nan"), device=DEV, dtype=torch.bfloat16)
    ops.conv_dgrad(dy, wt, dx, g, accumulate=True, acc_src=(src, bits))
    ref = torch.where(y > 0, src, torch.zeros_like(src))
    ops.conv_dgrad(dy, wt, ref, g, accumulate=True)
    torch.cuda.synchronize()
    assert torch.equal(dx, ref)
    cpu = torch.empty(B, H, H, C, dtype=torch.bfloat16)
    ops.conv_dgrad(dy.cpu(), wt.cpu(), cpu, g, accumulate=True, acc_src=(src.cpu(), bits.cpu()))
    assert (cpu.float() - dx.cpu().float()).abs().max().item() <= 2e-2 * dx.float().abs().max().item()

