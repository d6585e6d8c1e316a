"""Whole-image LDS convolution kernels (imgconv / imgwgrad) vs the fp32 reference."""
import pytest
import torch
import torch.nn.functional as F

import dtfe.ops as ops

DEV = "cuda"


def _rel(a, b):
    return ((a.float() - b.float()).abs().max() / (b.float().abs().max() + 1e-6)).item()


def test_flip_formulation_is_the_data_gradient_cpu():
    """imgconv(flip_taps, pad'=K-1-pad) over dY with Wt[cin][tap][cout] == dX of the conv (CPU, fp64-ish)."""
    torch.manual_seed(0)
    B, H, C, CO, K, pad = 2, 14, 8, 16, 5, 2
    x = torch.randn(B, C, H, H, requires_grad=True)
    w = torch.randn(CO, C, K, K)
    y = F.conv2d(x, w, padding=pad)
    gy = torch.randn_like(y)
    y.backward(gy)
    wt = w.permute(1, 2, 3, 0).contiguous()  # [cin][kh][kw][cout]
    out = torch.empty(B, H, H, C)
    ops.imgconv(wt, out, B=B, SH=H, SW=H, CS=CO, OH=H, OW=H, N=C, KH=K, KW=K, pad=K - 1 - pad,
                src=gy.permute(0, 2, 3, 1).contiguous(), flip_taps=True)
    assert torch.allclose(out, x.grad.permute(0, 2, 3, 1), atol=1e-4)


CASES = [  # (B, SH, CS, N, K, stride, pad, pool)
    (3, 14, 32, 64, 5, 1, 2, True),     # MNIST conv2 fwd
    (2, 32, 16, 16, 3, 1, 1, False),    # ResNet-20 stage 1
    (2, 32, 16, 32, 3, 2, 1, False),    # ResNet-20 downsample
    (2, 8, 64, 64, 3, 1, 1, False),     # ResNet-20 stage 3
    (3, 28, 1, 32, 5, 1, 2, True),      # MNIST conv1 fwd (1-channel tap-packed kernel)
    (2, 28, 1, 16, 3, 2, 1, False),     # 1-channel, strided, N=16
]


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES)
def test_imgconv_fwd(case):
    B, SH, CS, N, K, s, pad, pool = case
    OH = (SH + 2 * pad - K) // s + 1
    torch.manual_seed(1)
    x = torch.randn(B, SH, SH, CS).to(DEV, torch.bfloat16)
    w = (torch.randn(N, K, K, CS) * 0.1).to(DEV, torch.bfloat16)
    bias = torch.randn(N, device=DEV)
    shp = (B, OH // 2, OH // 2, N) if pool else (B, OH, OH, N)
    y = torch.empty(shp, device=DEV, dtype=torch.bfloat16)
    am = torch.empty(shp, device=DEV, dtype=torch.uint8) if pool else None
    kw = dict(B=B, SH=SH, SW=SH, CS=CS, OH=OH, OW=OH, N=N, KH=K, KW=K, stride=s, pad=pad, act=ops.ACT_RELU, pool=pool)
    ops.imgconv(w, y, src=x, bias=bias, argmax=am, **kw)
    yr = torch.empty(shp)
    amr = torch.empty(shp, dtype=torch.uint8) if pool else None
    ops.imgconv(w.cpu(), yr, src=x.cpu(), bias=bias.cpu(), argmax=amr, **kw)
    assert _rel(y.cpu(), yr) < 2e-2
    if pool:
        pos = yr > 0.05
        assert (am.cpu()[pos] == amr[pos]).float().mean().item() > 0.97


@pytest.mark.gpu
def test_imgconv_dgrad_unpool_source_and_mask():
    torch.manual_seed(2)
    B, H, CIN, COUT, K = 3, 14, 32, 64, 5
    dp = torch.randn(B, 7, 7, COUT).to(DEV, torch.bfloat16)
    am = torch.randint(0, 4, (B, 7, 7, COUT), dtype=torch.uint8).to(DEV)
    wt = (torch.randn(CIN, K, K, COUT) * 0.1).to(DEV, torch.bfloat16)
    mask = torch.randn(B, H, H, CIN).to(DEV, torch.bfloat16)
    y = torch.empty(B, H, H, CIN, device=DEV, dtype=torch.bfloat16)
    kw = dict(B=B, SH=H, SW=H, CS=COUT, OH=H, OW=H, N=CIN, KH=K, KW=K, pad=K - 1 - 2, flip_taps=True)
    ops.imgconv(wt, y, src_pooled=dp, src_argmax=am, relu_mask=mask, **kw)
    yr = torch.empty(B, H, H, CIN)
    ops.imgconv(wt.cpu(), yr, src_pooled=dp.cpu(), src_argmax=am.cpu(), relu_mask=mask.cpu(), **kw)
    assert _rel(y.cpu(), yr) < 2e-2
    assert float(y.cpu()[mask.cpu() <= 0].abs().max()) == 0.0


PERSIST_CASES = [  # B > 256 so persistent workgroups loop over several images
    (300, 14, 32, 64, 5, 1, 2, True),   # MNIST conv2 fwd
    (300, 32, 16, 16, 3, 1, 1, False),  # ResNet-20 stage 1
    (270, 16, 32, 32, 3, 2, 1, False),  # strided
    (300, 8, 64, 64, 3, 1, 1, False),   # ResNet-20 stage 3
    (300, 28, 1, 32, 5, 1, 2, True),    # MNIST conv1 (shifted-copy kernel, B >= 256)
]


@pytest.mark.gpu
@pytest.mark.parametrize("case", PERSIST_CASES)
def test_imgconv_persistent_fwd(case):
    test_imgconv_fwd(case)


@pytest.mark.gpu
def test_imgconv_persistent_dgrad_unpool_source_and_mask():
    torch.manual_seed(4)
    B, H, CIN, COUT, K = 300, 14, 32, 64, 5
    dp = torch.randn(B, 7, 7, COUT).to(DEV, torch.bfloat16)
    am = torch.randint(0, 4, (B, 7, 7, COUT), dtype=torch.uint8).to(DEV)
    wt = (torch.randn(CIN, K, K, COUT) * 0.1).to(DEV, torch.bfloat16)
    mask = torch.randn(B, H, H, CIN).to(DEV, torch.bfloat16)
    y = torch.empty(B, H, H, CIN, device=DEV, dtype=torch.bfloat16)
    kw = dict(B=B, SH=H, SW=H, CS=COUT, OH=H, OW=H, N=CIN, KH=K, KW=K, pad=K - 1 - 2, flip_taps=True)
    ops.imgconv(wt, y, src_pooled=dp, src_argmax=am, relu_mask=mask, **kw)
    yr = torch.empty(B, H, H, CIN)
    ops.imgconv(wt.cpu(), yr, src_pooled=dp.cpu(), src_argmax=am.cpu(), relu_mask=mask.cpu(), **kw)
    assert _rel(y.cpu(), yr) < 2e-2
    assert float(y.cpu()[mask.cpu() <= 0].abs().max()) == 0.0


@pytest.mark.gpu
@pytest.mark.parametrize("H,C", [(32, 16), (16, 32), (8, 64)])
def test_imgconv_persistent_dgrad_relu_mask_resnet20(H, C):
    """ResNet-20 data gradient (plain source, ReLU'-mask from a bf16 tensor): the LDS-staged
    epilogue applies the mask from 16-B loads at store time."""
    torch.manual_seed(6)
    B, K = 300, 3
    dy = torch.randn(B, H, H, C).to(DEV, torch.bfloat16)
    wt = (torch.randn(C, K, K, C) * 0.1).to(DEV, torch.bfloat16)
    mask = torch.randn(B, H, H, C).to(DEV, torch.bfloat16)
    mask[0, 0, 0, :4] = float("nan")
    mask[0, 0, 1, :4] = float("inf")
    kw = dict(B=B, SH=H, SW=H, CS=C, OH=H, OW=H, N=C, KH=K, KW=K, pad=1, flip_taps=True)
    y = torch.empty(B, H, H, C, device=DEV, dtype=torch.bfloat16)
    ops.imgconv(wt, y, src=dy, relu_mask=mask, **kw)
    yr = torch.empty(B, H, H, C)
    ops.imgconv(wt.cpu(), yr, src=dy.cpu(), relu_mask=mask.cpu(), **kw)
    assert _rel(y.cpu(), yr) < 2e-2
    keep = mask.cpu().float() > 0
    assert float(y.cpu()[~keep].abs().max()) == 0.0
    assert torch.equal(y.cpu()[0, 0, 1, :4], yr[0, 0, 1, :4].bfloat16())


WG_CASES = [  # (B, SH, CS, N, K, stride, pad, pooled_dy)
    (5, 14, 32, 64, 5, 1, 2, True),     # MNIST conv2 (dY = un-pooled dP2)
    (3, 32, 16, 16, 3, 1, 1, False),
    (3, 32, 16, 32, 3, 2, 1, False),
    (6, 8, 64, 64, 3, 1, 1, False),
    (5, 28, 1, 32, 5, 1, 2, True),      # MNIST conv1 (1-channel tap-packed kernel, dY = un-pooled dP1)
    (3, 28, 1, 64, 3, 2, 1, False),     # 1-channel, strided, N=64
    (7, 12, 1, 16, 5, 1, 0, False),     # 1-channel, valid padding, OW=8
]


@pytest.mark.gpu
@pytest.mark.parametrize("case", WG_CASES)
def test_imgwgrad(case):
    B, SH, CS, N, K, s, pad, pooled = case
    OH = (SH + 2 * pad - K) // s + 1
    torch.manual_seed(3)
    x = torch.randn(B, SH, SH, CS).to(DEV, torch.bfloat16)
    kw = dict(B=B, SH=SH, SW=SH, CS=CS, OH=OH, OW=OH, N=N, KH=K, KW=K, stride=s, pad=pad, scale=0.5)
    dw = torch.zeros(N, K, K, CS, device=DEV)
    db = torch.zeros(N, device=DEV)
    dwr, dbr = torch.zeros(N, K, K, CS), torch.zeros(N)
    if pooled:
        dp = torch.randn(B, OH // 2, OH // 2, N).to(DEV, torch.bfloat16)
        am = torch.randint(0, 4, dp.shape, dtype=torch.uint8).to(DEV)
        ops.imgwgrad(x, dw, db, dy_pooled=dp, dy_argmax=am, **kw)
        ops.imgwgrad(x.cpu(), dwr, dbr, dy_pooled=dp.cpu(), dy_argmax=am.cpu(), **kw)
    else:
        dy = torch.randn(B, OH, OH, N).to(DEV, torch.bfloat16)
        ops.imgwgrad(x, dw, db, dy=dy, **kw)
        ops.imgwgrad(x.cpu(), dwr, dbr, dy=dy.cpu(), **kw)
    assert _rel(dw.cpu(), dwr) < 1e-2
    assert _rel(db.cpu(), dbr) < 1e-2


PERSIST_WG_CASES = [  # B >= 128: persistent register-accumulating kernel
    (300, 14, 32, 64, 5, 1, 2, True),   # MNIST conv2 (dY = un-pooled dP2)
    (300, 16, 32, 32, 3, 1, 1, False),
    (260, 8, 64, 64, 3, 1, 1, False),
    (300, 32, 16, 16, 3, 1, 1, False),
    (200, 16, 16, 32, 3, 2, 1, False),  # strided
    (300, 28, 1, 32, 5, 1, 2, True),    # MNIST conv1 (shifted-copy kernel + partial-sum reduce)
]


@pytest.mark.gpu
@pytest.mark.parametrize("case", PERSIST_WG_CASES)
def test_imgwgrad_persistent(case):
    test_imgwgrad(case)


@pytest.mark.gpu
@pytest.mark.parametrize("case", [(96, 16, 32, 16, 3, 2, 1), (80, 8, 64, 32, 3, 2, 1)])
def test_imgconv_dilated_dgrad_of_strided_conv(case):
    """dX of a stride-2 conv = stride-1 flipped-tap conv over dY dilated by 2 (persistent kernel)."""
    B, OHs, COUT, CIN, K, s, pad = case
    H = OHs * s
    torch.manual_seed(5)
    dy = torch.randn(B, OHs, OHs, COUT).to(DEV, torch.bfloat16)
    wt = (torch.randn(CIN, K, K, COUT) * 0.1).to(DEV, torch.bfloat16)
    kw = dict(B=B, SH=OHs, SW=OHs, CS=COUT, OH=H, OW=H, N=CIN, KH=K, KW=K, stride=1, pad=K - 1 - pad,
              flip_taps=True, dil=s)
    y = torch.empty(B, H, H, CIN, device=DEV, dtype=torch.bfloat16)
    ops.imgconv(wt, y, src=dy, **kw)
    # oracle: autograd dX of the strided conv
    x = torch.zeros(B, CIN, H, H, requires_grad=True)
    w = wt.float().cpu().permute(3, 0, 1, 2)  # Wt[cin][kh][kw][cout] -> W[cout][cin][kh][kw]
    out = torch.nn.functional.conv2d(x, w, stride=s, padding=pad)
    out.backward(dy.float().cpu().permute(0, 3, 1, 2))
    assert _rel(y.cpu(), x.grad.permute(0, 2, 3, 1)) < 2e-2


@pytest.mark.gpu
@pytest.mark.parametrize("cs", [2, 3])
def test_few_channel_conv_fwd_wgrad(cs):
    """Tap-packed network-input kernels with CS = 2, 3 (CIFAR stem: 3x3x3 = 27 taps)."""
    B, H, N, K = 70, 32, 16, 3
    torch.manual_seed(6)
    x = torch.randn(B, H, H, cs).to(DEV, torch.bfloat16)
    w = (torch.randn(N, K, K, cs) * 0.2).to(DEV, torch.bfloat16)
    kw = dict(B=B, SH=H, SW=H, CS=cs, OH=H, OW=H, N=N, KH=K, KW=K, stride=1, pad=1)
    y = torch.empty(B, H, H, N, device=DEV, dtype=torch.bfloat16)
    ops.imgconv(w, y, src=x, **kw)
    yr = torch.empty(B, H, H, N)
    ops.imgconv(w.cpu(), yr, src=x.cpu(), **kw)
    assert _rel(y.cpu(), yr) < 2e-2
    dy = torch.randn(B, H, H, N).to(DEV, torch.bfloat16)
    dw, dwr = torch.zeros(N, K, K, cs, device=DEV), torch.zeros(N, K, K, cs)
    ops.imgwgrad(x, dw, None, dy=dy, **kw)
    ops.imgwgrad(x.cpu(), dwr, None, dy=dy.cpu(), **kw)
    assert _rel(dw.cpu(), dwr) < 1e-2



@pytest.mark.gpu
@pytest.mark.parametrize("B,H,CIN,COUT,s", [(256, 32, 16, 16, 1), (300, 16, 32, 32, 1), (256, 8, 64, 64, 1),
                                            (256, 32, 16, 32, 2), (130, 16, 32, 64, 2)])
def test_imgconv_shortcut_grad_fused(B, H, CIN, COUT, s):
    """Data gradient with the option-A shortcut gradient added in the epilogue == imgconv followed
    by shortcut_grad_add, bit for bit (stride 1 and the stride-2 dilated form)."""
    torch.manual_seed(9)
    OH = H // s
    dy = torch.randn(B, OH, OH, COUT).to(DEV, torch.bfloat16)
    wt = (torch.randn(CIN, 3, 3, COUT) * 0.1).to(DEV, torch.bfloat16)
    g = torch.randn(B, OH, OH, COUT).to(DEV, torch.bfloat16)
    geom = dict(B=B, SH=OH, SW=OH, CS=COUT, OH=H, OW=H, N=CIN, KH=3, KW=3, stride=1, pad=1, dil=s)
    ref = torch.empty(B, H, H, CIN, device=DEV, dtype=torch.bfloat16)
    ops.imgconv(wt, ref, src=dy, flip_taps=True, **geom)
    ops.shortcut_grad_add(g, ref, s)
    dx = torch.empty_like(ref)
    assert ops.imgconv_shortcut(wt, dx, g, s, src=dy, **geom)
    assert torch.equal(dx, ref)


def test_imgconv_shortcut_cpu_oracle():
    torch.manual_seed(10)
    B, H, C = 2, 8, 16
    dy = torch.randn(B, H // 2, H // 2, 2 * C).bfloat16()
    wt = (torch.randn(C, 3, 3, 2 * C) * 0.1).bfloat16()
    g = torch.randn(B, H // 2, H // 2, 2 * C).bfloat16()
    geom = dict(B=B, SH=H // 2, SW=H // 2, CS=2 * C, OH=H, OW=H, N=C, KH=3, KW=3, stride=1, pad=1, dil=2)
    dx = torch.empty(B, H, H, C, dtype=torch.bfloat16)
    assert ops.imgconv_shortcut(wt, dx, g, 2, src=dy, **geom)
    ref = torch.empty_like(dx)
    ops.imgconv(wt, ref, src=dy, flip_taps=True, **geom)
    ops.shortcut_grad_add(g, ref, 2)
    assert torch.equal(dx, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("case", [(256, 32, 16, 16, 3, 1, 1), (256, 32, 16, 32, 3, 2, 1), (300, 16, 32, 32, 3, 1, 1),
                                  (256, 8, 64, 64, 3, 1, 1), (130, 16, 16, 32, 3, 2, 1)])
def test_imgwgrad_persistent_kgroups(case):
    """Weight gradient without a bias gradient (ResNet convs): the k-group wave split (KG = 8 / 4 for
    9 / 18 column tiles) and the 5-tile column groups of the 64-channel layers vs the fp32 reference,
    and equal to the wave-per-column-tiles kernel (DTFE_DIAG iwk=1 path) to fp32 rounding."""
    B, SH, CS, N, K, s, pad = case
    OH = (SH + 2 * pad - K) // s + 1
    torch.manual_seed(11)
    x = torch.randn(B, SH, SH, CS).to(DEV, torch.bfloat16)
    dy = torch.randn(B, OH, OH, N).to(DEV, torch.bfloat16)
    kw = dict(B=B, SH=SH, SW=SH, CS=CS, OH=OH, OW=OH, N=N, KH=K, KW=K, stride=s, pad=pad, scale=0.5)
    dw = torch.zeros(N, K, K, CS, device=DEV)
    ops.imgwgrad(x, dw, None, dy=dy, **kw)
    dwr = torch.zeros(N, K, K, CS)
    ops.imgwgrad(x.cpu(), dwr, None, dy=dy.cpu(), **kw)
    assert _rel(dw.cpu(), dwr) < 1e-2
    dw2 = torch.zeros_like(dw)
    ops.imgwgrad(x, dw2, None, dy=dy, **kw)  # a second launch (workspace / LDS reuse)
    assert torch.equal(dw, dw2)


@pytest.mark.gpu
@pytest.mark.parametrize("B,H,C", [(256, 32, 16), (200, 16, 32), (160, 8, 64)])
def test_imgconv_bn_src_on_load_matches_materialised(B, H, C):
    """A BN + ReLU formed on the whole-image conv's source while staging it (bn_src) == bn_apply's
    materialised output fed to the conv: forward output, saved mean / invstd, moving averages and
    the weight gradient bit for bit."""
    torch.manual_seed(12)
    x = (torch.randn(B, H, H, C) * 2 + 0.5).to(DEV, torch.bfloat16)
    stats = torch.zeros(2 * C, device=DEV)
    ops.bn_stats(x, stats)
    gamma = torch.rand(C, device=DEV) + 0.5
    beta = torch.randn(C, device=DEV) * 0.1
    mm0, mv0 = torch.randn(C, device=DEV), torch.rand(C, device=DEV) + 0.5
    h = torch.empty_like(x)
    ref = [torch.zeros(C, device=DEV), torch.zeros(C, device=DEV), mm0.clone(), mv0.clone()]
    ops.bn_apply(x, stats, gamma, beta, h, mean=ref[0], invstd=ref[1], moving_mean=ref[2], moving_var=ref[3],
                 eps=1e-3, momentum=0.99)
    w = (torch.randn(C, 3, 3, C) * 0.1).to(DEV, torch.bfloat16)
    kw = dict(B=B, SH=H, SW=H, CS=C, OH=H, OW=H, N=C, KH=3, KW=3, stride=1, pad=1)
    y_ref = torch.empty_like(x)
    ops.imgconv(w, y_ref, src=h, **kw)
    got = [torch.zeros(C, device=DEV), torch.zeros(C, device=DEV), mm0.clone(), mv0.clone()]
    y = torch.empty_like(x)
    ops.imgconv(w, y, src=x, bn_src=[stats, gamma, beta] + got, bn_eps=1e-3, bn_momentum=0.99, bn_save=True, **kw)
    assert torch.equal(y, y_ref)
    for a, b in zip(got, ref):
        assert torch.equal(a, b)
    dy = torch.randn(B, H, H, C).to(DEV, torch.bfloat16)
    wk = {k: v for k, v in kw.items()}
    dw_ref, dw = torch.zeros(C, 3, 3, C, device=DEV), torch.zeros(C, 3, 3, C, device=DEV)
    ops.imgwgrad(h, dw_ref, None, dy=dy, **wk)
    ops.imgwgrad(x, dw, None, dy=dy, bn_src=[stats, gamma, beta] + got, bn_eps=1e-3, **wk)
    assert torch.equal(dw, dw_ref)


def test_imgconv_bn_src_cpu_oracle():
    torch.manual_seed(13)
    B, H, C = 2, 8, 16
    x = torch.randn(B, H, H, C).bfloat16()
    stats = torch.zeros(2 * C)
    ops.bn_stats(x, stats)
    gamma, beta = torch.rand(C) + 0.5, torch.randn(C) * 0.1
    h = torch.empty_like(x)
    ops.bn_apply(x, stats, gamma, beta, h, eps=1e-3, momentum=0.99)
    w = (torch.randn(C, 3, 3, C) * 0.1).bfloat16()
    kw = dict(B=B, SH=H, SW=H, CS=C, OH=H, OW=H, N=C, KH=3, KW=3, stride=1, pad=1)
    y_ref, y = torch.empty_like(x), torch.empty_like(x)
    ops.imgconv(w, y_ref, src=h, **kw)
    z = torch.zeros(C)
    ops.imgconv(w, y, src=x, bn_src=[stats, gamma, beta, z, z.clone(), z.clone(), z.clone() + 1], **kw)
    assert torch.equal(y, y_ref)


@pytest.mark.gpu
def test_imgwgrad_deferred_reduces_grouped_flush():
    """Weight gradients whose partial-slab reduces are queued (defer=True, own workspaces) and summed
    by ONE grouped launch (ops.wgrad_flush) == the per-call reduce, bit for bit."""
    torch.manual_seed(16)
    shapes = [(256, 32, 16, 16, 1), (256, 16, 32, 32, 1), (256, 8, 64, 64, 1), (256, 32, 16, 32, 2)]
    ref, got, ws = [], [], []
    args = []
    for B, SH, CS, N, s in shapes:
        OH = (SH + 2 - 3) // s + 1
        x = torch.randn(B, SH, SH, CS).to(DEV, torch.bfloat16)
        dy = torch.randn(B, OH, OH, N).to(DEV, torch.bfloat16)
        kw = dict(B=B, SH=SH, SW=SH, CS=CS, OH=OH, OW=OH, N=N, KH=3, KW=3, stride=s, pad=1)
        args.append((x, dy, kw))
        r = torch.zeros(N, 3, 3, CS, device=DEV)
        ops.imgwgrad(x, r, None, dy=dy, **kw)
        ref.append(r)
    for x, dy, kw in args:
        g = torch.zeros(kw["N"], 3, 3, kw["CS"], device=DEV)
        w = torch.empty(ops.wgrad_ws_floats(kw["N"], 9 * kw["CS"]), device=DEV)
        ops.imgwgrad(x, g, None, dy=dy, workspace=w, defer=True, **kw)
        got.append(g)
        ws.append(w)
    assert ops.wgrad_flush() == len(shapes)
    torch.cuda.synchronize()
    for a, b in zip(got, ref):
        assert torch.equal(a, b)
    assert ops.wgrad_flush() == 0
