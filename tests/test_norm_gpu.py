"""BatchNorm / shortcut / pooling HIP kernels vs the fp32 reference path of the same ops."""
import pytest
import torch

import dtfe  # noqa: F401
from dtfe import ops

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    return ((a.float().cpu() - b.float().cpu()).abs().max() / (b.float().cpu().abs().max() + 1e-6)).item()


@pytest.mark.parametrize("shape,res_shape,rstride,from_x", [
    ((8, 16, 16, 32), None, 1, False),
    ((8, 16, 16, 32), None, 1, True),             # ReLU mask recomputed from x (no y read)
    ((8, 16, 16, 32), (8, 16, 16, 32), 1, False),  # identity shortcut
    ((8, 8, 8, 64), (8, 16, 16, 32), 2, False),   # option A: subsample + zero channels
    ((4, 7, 7, 2048), None, 1, False),            # ResNet-50 widest layer
    ((4, 7, 7, 2048), None, 1, True),
    ((3, 17, 19, 64), None, 1, True),             # row count with ragged unroll tails
    ((16, 56, 56, 64), None, 1, False),           # many row batches per stats thread
])
def test_bn_forward_backward(shape, res_shape, rstride, from_x):
    torch.manual_seed(0)
    C = shape[-1]
    x = (torch.randn(*shape) * 2 + 3).to(torch.bfloat16)  # |mean| >> std: the shifted statistics matter
    res = torch.randn(*res_shape).to(torch.bfloat16) if res_shape else None
    gamma, beta = torch.rand(C) + 0.5, torch.randn(C)
    dy = torch.randn(*shape).to(torch.bfloat16)
    out = {}
    for dev in ("cpu", DEV):
        st = torch.zeros(2 * C, device=dev)
        mean, inv = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
        mm, mv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
        y = torch.empty(*shape, device=dev, dtype=torch.bfloat16)
        xd = x.to(dev)
        ops.bn_stats(xd, st)
        ops.bn_apply(xd, st, gamma.to(dev), beta.to(dev), y, mean=mean, invstd=inv, moving_mean=mm, moving_var=mv,
                     act=ops.ACT_RELU, res=res.to(dev) if res is not None else None, rstride=rstride)
        st2 = torch.zeros(2 * C, device=dev)
        dx = torch.empty(*shape, device=dev, dtype=torch.bfloat16)
        dres = torch.empty(*shape, device=dev, dtype=torch.bfloat16)
        dg, db = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
        ym, bt = (None, beta.to(dev)) if from_x else (y, None)
        ops.bn_bwd_stats(dy.to(dev), ym, xd, mean, inv, st2, ops.ACT_RELU, gamma=gamma.to(dev), beta=bt)
        ops.bn_bwd_apply(dy.to(dev), ym, xd, mean, inv, gamma.to(dev), st2, dx, act=ops.ACT_RELU, dres=dres,
                         dgamma=dg, dbeta=db, beta=bt)
        out[dev] = dict(y=y, mean=mean, inv=inv, mm=mm, mv=mv, dx=dx, dres=dres, dg=dg, db=db)
    c, g = out["cpu"], out[DEV]
    for k in ("mean", "inv", "mm", "mv", "dg", "db"):
        assert _rel(g[k], c[k]) < 2e-3, k
    for k in ("y", "dx", "dres"):
        assert _rel(g[k], c[k]) < 2e-2, k


@pytest.mark.parametrize("shape,res_shape,rstride", [
    ((8, 16, 16, 32), (8, 16, 16, 32), 1),   # identity shortcut
    ((8, 8, 8, 64), (8, 16, 16, 32), 2),     # option A
    ((4, 7, 7, 2048), (4, 7, 7, 2048), 1),   # ResNet-50 widest block output
    ((3, 17, 19, 64), (3, 17, 19, 64), 1),   # ragged row count
])
def test_bn_relu_bitmask_matches_y(shape, res_shape, rstride):
    """bn_apply(mask_out=...) writes the 1-bit ReLU mask of its output (= the host-side
    relu_bits(y) of the stored values, bit for bit); the backward ops given that mask produce the
    masked gradient (dres) bit for bit as with the bf16 output y, and the same statistics / dx up to
    the order of the statistics kernel's per-workgroup float atomics."""
    torch.manual_seed(3)
    C = shape[-1]
    x = (torch.randn(*shape, device=DEV) * 2 + 1).to(torch.bfloat16)
    res = torch.randn(*res_shape, device=DEV).to(torch.bfloat16)
    gamma, beta = torch.rand(C, device=DEV) + 0.5, torch.randn(C, device=DEV)
    dy = torch.randn(*shape, device=DEV).to(torch.bfloat16)
    st = torch.zeros(2 * C, device=DEV)
    mean, inv = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
    y = torch.empty(*shape, device=DEV, dtype=torch.bfloat16)
    bits = torch.full((x.numel() // 8,), 0xA5, device=DEV, dtype=torch.uint8)
    ops.bn_stats(x, st)
    ops.bn_apply(x, st, gamma, beta, y, mean=mean, invstd=inv, act=ops.ACT_RELU, res=res, rstride=rstride,
                 mask_out=bits)
    torch.cuda.synchronize()
    assert torch.equal(bits.cpu(), ops.relu_bits(y.cpu()))
    outs = []
    for ym in (y, bits):
        st2 = torch.zeros(2 * C, device=DEV)
        dx = torch.empty(*shape, device=DEV, dtype=torch.bfloat16)
        dres = torch.empty(*shape, device=DEV, dtype=torch.bfloat16)
        dg, db = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
        ops.bn_bwd_stats(dy, ym, x, mean, inv, st2, ops.ACT_RELU, gamma=gamma)
        ops.bn_bwd_apply(dy, ym, x, mean, inv, gamma, st2, dx, act=ops.ACT_RELU, dres=dres, dgamma=dg, dbeta=db)
        outs.append((st2, dx, dres, dg, db))
    torch.cuda.synchronize()
    (s_y, dx_y, dr_y, dg_y, db_y), (s_b, dx_b, dr_b, dg_b, db_b) = outs
    assert torch.equal(dr_y, dr_b)
    for u, v in ((s_y, s_b), (dg_y, dg_b), (db_y, db_b)):
        assert torch.allclose(u, v, rtol=1e-5, atol=1e-5 * float(u.abs().max()))
    assert _rel(dx_b, dx_y) < 1e-2
    # the CPU reference with the mask: same gradient as with y
    st3 = torch.zeros(2 * C)
    ops.bn_bwd_stats(dy.cpu(), bits.cpu(), x.cpu(), mean.cpu(), inv.cpu(), st3, ops.ACT_RELU)
    assert _rel(outs[0][0], st3) < 2e-3


def test_shortcut_grad_add_and_gap():
    torch.manual_seed(1)
    g = torch.randn(4, 8, 8, 64).to(torch.bfloat16)
    dx0 = torch.randn(4, 16, 16, 32).to(torch.bfloat16)
    a, b = dx0.clone(), dx0.clone().to(DEV)
    ops.shortcut_grad_add(g, a, 2)
    ops.shortcut_grad_add(g.to(DEV), b, 2)
    assert _rel(b, a) < 1e-2
    x = torch.randn(4, 8, 8, 64).to(torch.bfloat16)
    y1, y2 = torch.empty(4, 64, dtype=torch.bfloat16), torch.empty(4, 64, dtype=torch.bfloat16, device=DEV)
    ops.gap_fwd(x, y1)
    ops.gap_fwd(x.to(DEV), y2)
    assert _rel(y2, y1) < 1e-2
    d1, d2 = torch.empty(4, 8, 8, 64, dtype=torch.bfloat16), torch.empty(4, 8, 8, 64, dtype=torch.bfloat16, device=DEV)
    ops.gap_bwd(y1, d1)
    ops.gap_bwd(y1.to(DEV), d2)
    assert _rel(d2, d1) < 1e-2


@pytest.mark.parametrize("B,H,W,C", [(2, 112, 112, 64), (3, 7, 9, 64), (2, 15, 15, 32), (1, 9, 6, 128)])
def test_maxpool3(B, H, W, C):
    """Odd H / W exercise the backward's partial 2x2 input cells at the bottom / right edge."""
    torch.manual_seed(2)
    OH, OW = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    x = torch.randn(B, H, W, C).to(torch.bfloat16)
    ys, ams, dxs = [], [], []
    dy = torch.randn(B, OH, OW, C).to(torch.bfloat16)
    for dev in ("cpu", DEV):
        y = torch.empty(B, OH, OW, C, dtype=torch.bfloat16, device=dev)
        am = torch.empty(B, OH, OW, C, dtype=torch.uint8, device=dev)
        dx = torch.empty(B, H, W, C, dtype=torch.bfloat16, device=dev)
        ops.maxpool3_fwd(x.to(dev), y, am)
        ops.maxpool3_bwd(dy.to(dev), am, dx)
        ys.append(y.cpu()), ams.append(am.cpu()), dxs.append(dx.cpu())
    assert torch.equal(ys[0], ys[1])
    assert (ams[0] == ams[1]).float().mean() > 0.999
    assert _rel(dxs[1], dxs[0]) < 1e-2


@pytest.mark.gpu
@pytest.mark.parametrize("B,H,C,Cout,k", [(3, 14, 64, 128, 3), (64, 56, 64, 64, 1), (16, 28, 128, 256, 3)])
def test_conv_fwd_fused_bn_stats_match_separate_pass(B, H, C, Cout, k):
    """The implicit-GEMM forward's epilogue BatchNorm partials (per tile, two-stage fixed-order
    reduction) give the statistics the separate bn_stats pass computes from the stored output."""
    from dtfe import ops

    torch.manual_seed(3)
    x = torch.randn(B, H, H, C, device="cuda").to(torch.bfloat16)
    w = (torch.randn(Cout, k, k, C, device="cuda") * 0.05).to(torch.bfloat16)
    g = dict(B=B, H=H, W=H, C=C, Cout=Cout, OH=H, OW=H, KH=k, KW=k, stride=1, pad=(k - 1) // 2)
    y1 = torch.empty(B, H, H, Cout, device="cuda", dtype=torch.bfloat16)
    y2 = torch.empty_like(y1)
    s1 = torch.zeros(2 * Cout, device="cuda")
    s2 = torch.zeros(2 * Cout, device="cuda")
    ops.conv_fwd(x, w, None, y1, None, g, act=ops.ACT_NONE, stats=s1)
    ops.conv_fwd(x, w, None, y2, None, g, act=ops.ACT_NONE)
    ops.bn_stats(y2, s2)
    assert torch.equal(y1, y2)
    R = B * H * H
    # compare the derived mean / variance (the raw shifted sums are tiny when the shift is close)
    m1, m2 = s1[:Cout] / R, s2[:Cout] / R
    v1, v2 = s1[Cout:] / R - m1 * m1, s2[Cout:] / R - m2 * m2
    assert torch.allclose(m1, m2, rtol=1e-3, atol=1e-5)
    assert torch.allclose(v1, v2, rtol=1e-3, atol=1e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("B", [2, 5])
def test_stem_fwd_fused_bn_stats_match_separate_pass(B):
    """The ImageNet stem (7x7/2, 3->64) forward emits per-block BatchNorm partials from its epilogue
    (two fold launches instead of a pass over y): the statistics equal the separate bn_stats pass."""
    torch.manual_seed(4)
    x = (torch.rand(B, 224, 224, 3, device="cuda") * 2 - 0.5).to(torch.bfloat16)
    w = (torch.randn(64, 7, 7, 3, device="cuda") * 0.1).to(torch.bfloat16)
    g = dict(B=B, H=224, W=224, C=3, Cout=64, OH=112, OW=112, KH=7, KW=7, stride=2, pad=3)
    y1 = torch.empty(B, 112, 112, 64, device="cuda", dtype=torch.bfloat16)
    y2 = torch.empty_like(y1)
    s1, s2 = torch.zeros(128, device="cuda"), torch.zeros(128, device="cuda")
    ops.conv_fwd(x, w, None, y1, None, g, act=ops.ACT_NONE, stats=s1)
    ops.conv_fwd(x, w, None, y2, None, g, act=ops.ACT_NONE)
    ops.bn_stats(y2, s2)
    assert torch.equal(y1, y2)
    R = B * 112 * 112
    m1, m2 = s1[:64] / R, s2[:64] / R
    v1, v2 = s1[64:] / R - m1 * m1, s2[64:] / R - m2 * m2
    assert torch.allclose(m1, m2, rtol=1e-3, atol=1e-5)
    assert torch.allclose(v1, v2, rtol=1e-3, atol=1e-6)


@pytest.mark.parametrize("shape", [(4, 112, 112, 64), (3, 17, 13, 16), (2, 9, 10, 256)])
def test_bn_relu_pool3_bitwise_vs_apply_then_pool(shape):
    """bn_relu_pool3 (ResNet-50 stem: BN + ReLU + 3x3/s2 max pool in one pass) == bn_apply followed
    by maxpool3_fwd, bit for bit: pooled values, argmax, saved mean / invstd and moving averages.
    Odd spatial sizes exercise the padded last window row / column."""
    torch.manual_seed(5)
    B, H, W, C = shape
    x = (torch.randn(B, H, W, C) * 1.7 + 0.4).to(DEV, torch.bfloat16)
    g = (torch.rand(C) + 0.5).to(DEV)
    bt = (torch.randn(C) * 0.3).to(DEV)
    stats = torch.zeros(2 * C, device=DEV)
    ops.bn_stats(x, stats)
    OH, OW = (H + 1) // 2, (W + 1) // 2
    outs = []
    for fused in (False, True):
        mean, inv = torch.empty(C, device=DEV), torch.empty(C, device=DEV)
        mm, mv = torch.full((C,), 0.1, device=DEV), torch.full((C,), 0.9, device=DEV)
        y = torch.full((B, OH, OW, C), float("nan"), device=DEV, dtype=torch.bfloat16)
        am = torch.full((B, OH, OW, C), 255, device=DEV, dtype=torch.uint8)
        kw = dict(mean=mean, invstd=inv, moving_mean=mm, moving_var=mv, eps=1e-5, momentum=0.9)
        if fused:
            ops.bn_relu_pool3(x, stats, g, bt, y, am, **kw)
        else:
            h = torch.empty_like(x)
            ops.bn_apply(x, stats, g, bt, h, act=ops.ACT_RELU, **kw)
            ops.maxpool3_fwd(h, y, am)
        outs.append((y, am, mean, inv, mm, mv))
    for a, b in zip(*outs):
        assert torch.equal(a, b)


@pytest.mark.parametrize("shape", [(4, 112, 112, 64), (3, 17, 13, 16), (2, 9, 10, 256)])
def test_pool3_bn_bwd_matches_pool_bwd_then_bn_bwd(shape):
    """pool3_bn_bwd (max-pool backward fused into the stem BN's backward, ReLU mask from x) vs
    maxpool3_bwd + bn_bwd_stats + bn_bwd_apply: statistics to fp32 summation-order tolerance (both
    reduce with atomics), dx / dgamma / dbeta bit-identical given the same statistics."""
    torch.manual_seed(6)
    B, H, W, C = shape
    OH, OW = (H + 1) // 2, (W + 1) // 2
    x = (torch.randn(B, H, W, C) * 1.3 + 0.2).to(DEV, torch.bfloat16)
    g = (torch.rand(C) + 0.5).to(DEV)
    bt = (torch.randn(C) * 0.3).to(DEV)
    st = torch.zeros(2 * C, device=DEV)
    ops.bn_stats(x, st)
    mean, inv = torch.empty(C, device=DEV), torch.empty(C, device=DEV)
    pool = torch.empty(B, OH, OW, C, device=DEV, dtype=torch.bfloat16)
    am = torch.empty(B, OH, OW, C, device=DEV, dtype=torch.uint8)
    ops.bn_relu_pool3(x, st, g, bt, pool, am, mean=mean, invstd=inv, eps=1e-5, momentum=0.9)
    dp = torch.randn(B, OH, OW, C).to(DEV, torch.bfloat16)
    # reference: unpooled gradient, then the two BN backward passes
    d = torch.empty_like(x)
    ops.maxpool3_bwd(dp, am, d)
    s_ref = torch.zeros(2 * C, device=DEV)
    ops.bn_bwd_stats(d, None, x, mean, inv, s_ref, ops.ACT_RELU, gamma=g, beta=bt)
    s_f = torch.zeros(2 * C, device=DEV)
    dx_f = torch.full_like(x, float("nan"))
    dg_f, db_f = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
    ops.pool3_bn_bwd(dp, am, x, mean, inv, g, bt, s_f, dx_f, dgamma=dg_f, dbeta=db_f)
    assert torch.allclose(s_f, s_ref, rtol=1e-3, atol=1e-3 * float(s_ref.abs().max()))
    dx_r = torch.empty_like(x)
    dg_r, db_r = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
    ops.bn_bwd_apply(d, None, x, mean, inv, g, s_f, dx_r, act=ops.ACT_RELU, dgamma=dg_r, dbeta=db_r, beta=bt)
    assert torch.equal(dx_f, dx_r) and torch.equal(dg_f, dg_r) and torch.equal(db_f, db_r)


@pytest.mark.parametrize("shape", [(2, 14, 14, 256), (3, 5, 7, 64)])
def test_bn_apply_residual_bn_fold_bitwise(shape):
    """bn_apply(res=raw shortcut, res_bn=...) (a projection shortcut's BN folded into the residual
    apply) == the shortcut's own bn_apply(ACT_NONE) followed by the residual bn_apply: the output,
    its ReLU bit mask and both BNs' saved statistics / moving averages, bit for bit."""
    torch.manual_seed(9)
    B, H, W, C = shape
    x = (torch.randn(B, H, W, C) * 1.1 - 0.3).to(DEV, torch.bfloat16)
    zs = (torch.randn(B, H, W, C) * 0.7 + 0.5).to(DEV, torch.bfloat16)
    st, sst = torch.zeros(2 * C, device=DEV), torch.zeros(2 * C, device=DEV)
    ops.bn_stats(x, st)
    ops.bn_stats(zs, sst)
    g, bt = (torch.rand(C) + 0.5).to(DEV), (torch.randn(C) * 0.2).to(DEV)
    gs, bs = (torch.rand(C) + 0.5).to(DEV), (torch.randn(C) * 0.2).to(DEV)

    def bufs():
        return ([torch.empty(C, device=DEV) for _ in range(2)] + [torch.full((C,), 0.1, device=DEV),
                                                                 torch.full((C,), 0.9, device=DEV)])
    outs = []
    for fused in (False, True):
        m, i, mm, mv = bufs()
        rm, ri, rmm, rmv = bufs()
        y = torch.empty_like(x)
        bits = torch.empty(x.numel() // 8, device=DEV, dtype=torch.uint8)
        kw = dict(mean=m, invstd=i, moving_mean=mm, moving_var=mv, eps=1e-3, momentum=0.99, act=ops.ACT_RELU,
                  mask_out=bits)
        if fused:
            ops.bn_apply(x, st, g, bt, y, res=zs, res_bn=[sst, gs, bs, rm, ri, rmm, rmv], **kw)
        else:
            ys = torch.empty_like(zs)
            ops.bn_apply(zs, sst, gs, bs, ys, mean=rm, invstd=ri, moving_mean=rmm, moving_var=rmv, eps=1e-3,
                         momentum=0.99, act=ops.ACT_NONE)
            ops.bn_apply(x, st, g, bt, y, res=ys, **kw)
        outs.append((y, bits, m, i, mm, mv, rm, ri, rmm, rmv))
    for a, b in zip(*outs):
        assert torch.equal(a, b)


def test_bn_bwd_stats_dual_matches_two_passes():
    """bn_bwd_stats(res_bn=[x2, mean2, invstd2, stats2]) == two bn_bwd_stats passes sharing the
    bit-masked g (the second over x2), to fp32 summation-order tolerance."""
    torch.manual_seed(10)
    R, C = 3000, 256
    x = torch.randn(R, C).to(DEV, torch.bfloat16)
    x2 = (torch.randn(R, C) * 0.5 + 1).to(DEV, torch.bfloat16)
    dy = torch.randn(R, C).to(DEV, torch.bfloat16)
    y = torch.relu(torch.randn(R, C)).to(DEV, torch.bfloat16)
    bits = ops.relu_bits(y)
    mean, inv = (torch.randn(C) * 0.1).to(DEV), (torch.rand(C) + 0.5).to(DEV)
    m2, i2 = (torch.randn(C) * 0.1 + 1).to(DEV), (torch.rand(C) + 1.5).to(DEV)
    a, b = torch.zeros(2 * C, device=DEV), torch.zeros(2 * C, device=DEV)
    ops.bn_bwd_stats(dy, bits, x, mean, inv, a, ops.ACT_RELU)
    ops.bn_bwd_stats(dy, bits, x2, m2, i2, b, ops.ACT_RELU)
    a2, b2 = torch.zeros(2 * C, device=DEV), torch.zeros(2 * C, device=DEV)
    ops.bn_bwd_stats(dy, bits, x, mean, inv, a2, ops.ACT_RELU, res_bn=[x2, m2, i2, b2])
    for u, v in ((a, a2), (b, b2)):
        assert torch.allclose(u, v, rtol=1e-4, atol=1e-4 * float(u.abs().max()))
