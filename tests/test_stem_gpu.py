"""ImageNet stem kernels (csrc/kernels/stem.hip): 7x7/2 conv 3 -> 64, 224 -> 112, forward and weight
gradient against fp32 PyTorch on the same bf16 values (BASELINE.json config 5)."""
import pytest
import torch

from dtfe import ops

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _geom(B):
    return dict(B=B, H=224, W=224, C=3, Cout=64, OH=112, OW=112, KH=7, KW=7, stride=2, pad=3)


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12))


@pytest.mark.parametrize("B", [3, 260])
def test_stem_fwd_matches_conv2d(B):
    torch.manual_seed(0)
    x = torch.randn(B, 224, 224, 3, device=DEV).to(torch.bfloat16)
    w = (torch.randn(64, 7, 7, 3, device=DEV) * 0.1).to(torch.bfloat16)
    y = torch.empty(B, 112, 112, 64, device=DEV, dtype=torch.bfloat16)
    ops.conv_fwd(x, w, None, y, None, _geom(B), act=ops.ACT_NONE)
    ref = torch.nn.functional.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), stride=2,
                                     padding=3).permute(0, 2, 3, 1)
    assert _rel(y, ref) < 8e-3


@pytest.mark.parametrize("B", [3, 260])
def test_stem_wgrad_matches_conv2d_weight(B):
    torch.manual_seed(1)
    x = torch.randn(B, 224, 224, 3, device=DEV).to(torch.bfloat16)
    dy = (torch.randn(B, 112, 112, 64, device=DEV) * 0.1).to(torch.bfloat16)
    init = torch.randn(64, 7, 7, 3, device=DEV)
    dw = init.clone()
    ops.conv_wgrad(dy, x, dw, None, _geom(B), 0.5)
    ref = torch.nn.grad.conv2d_weight(x.float().permute(0, 3, 1, 2), (64, 3, 7, 7), dy.float().permute(0, 3, 1, 2),
                                      stride=2, padding=3).permute(0, 2, 3, 1)
    assert _rel(dw - init, 0.5 * ref) < 2e-3   # += semantics, fp32 accumulation
    dw2 = init.clone()
    ops.conv_wgrad(dy, x, dw2, None, _geom(B), 0.5)
    assert torch.equal(dw, dw2)                  # fixed-order reduction: bitwise reproducible
