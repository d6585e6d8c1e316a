"""Numerics of every HIP kernel against a plain-PyTorch fp32 reference (T3).

Asymmetric operands everywhere (A=I checks with asymmetric B catch C-write
transposes), odd sizes for masked tails, all operand layouts.
"""
import itertools

import pytest
import torch

import dtfe.ops as ops

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    return ((a.float() - b.float()).abs().max() / (b.float().abs().max() + 1e-6)).item()


def _operand(mat, mode, dtype):
    """Store logical [rows, K] matrix in the requested mode; return (tensor, ld)."""
    if mode == ops.KMAJ:
        t = mat.contiguous()
        return t.to(DEV, dtype), mat.shape[1]
    t = mat.t().contiguous()
    return t.to(DEV, dtype), mat.shape[0]


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("amode,bmode", list(itertools.product([0, 1], [0, 1])))
@pytest.mark.parametrize("tile", [0, 1, 2, 3, 4])
def test_gemm_modes_tiles(dtype, amode, bmode, tile):
    torch.manual_seed(0)
    M, N, K = 200, 136, 264
    A = torch.randn(M, K)
    B = torch.randn(N, K)
    At, lda = _operand(A, amode, dtype)
    Bt, ldb = _operand(B, bmode, dtype)
    out = torch.zeros(M, N, device=DEV, dtype=torch.float32)
    ops.gemm(At, Bt, out, M=M, N=N, K=K, amode=amode, lda=lda, bmode=bmode, ldb=ldb, tile=tile)
    ref = At.float().cpu() if amode == 0 else At.float().cpu().t()
    refb = Bt.float().cpu() if bmode == 0 else Bt.float().cpu().t()
    exp = ref @ refb.t()
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-5
    assert _rel(out.cpu(), exp) < tol


@pytest.mark.parametrize("amode,bmode", list(itertools.product([0, 1], [0, 1])))
@pytest.mark.parametrize("M,N,K", [(200, 136, 264), (257, 1, 256), (128, 784, 100), (17, 33, 1), (785, 256, 2049)])
def test_gemm_small_tile_exact_fp32(amode, bmode, M, N, K):
    """Small-layer fp32 kernel (tile 13): odd shapes, K not a multiple of 4/16, N = 1, K = 1."""
    torch.manual_seed(3)
    A = torch.randn(M, K)
    B = torch.randn(N, K)
    At, lda = _operand(A, amode, torch.float32)
    Bt, ldb = _operand(B, bmode, torch.float32)
    out = torch.full((M, N), float("nan"), device=DEV)
    ops.gemm(At, Bt, out, M=M, N=N, K=K, amode=amode, lda=lda, bmode=bmode, ldb=ldb, tile=ops.TILE_SMALL)
    exp = A.double() @ B.double().t()
    assert _rel(out.cpu().double(), exp) < 1e-5


def test_gemm_small_tile_ones_rows_and_aux():
    """Weight-gradient form: bias gradient through a ones row (A side and B side), act' epilogue."""
    torch.manual_seed(4)
    X, D = torch.randn(256, 100, device=DEV), torch.randn(256, 64, device=DEV)
    dw = torch.empty(100, 64, device=DEV)
    db = torch.empty(64, device=DEV)
    ops.gemm(X, D, dw, M=101, N=64, K=256, amode=ops.RMAJ, lda=100, bmode=ops.RMAJ, ldb=64, a_ones_row=100,
             bias_out=db, tile=ops.TILE_SMALL)
    assert _rel(dw.cpu(), X.cpu().t() @ D.cpu()) < 1e-5 and _rel(db.cpu(), D.cpu().sum(0)) < 1e-5
    dw2 = torch.empty(64, 100, device=DEV)
    db2 = torch.empty(64, device=DEV)
    ops.gemm(D, X, dw2, M=64, N=101, K=256, amode=ops.RMAJ, lda=64, bmode=ops.RMAJ, ldb=100, ldc=100,
             b_ones_row=100, bias_out=db2, tile=ops.TILE_SMALL)
    assert _rel(dw2.cpu(), D.cpu().t() @ X.cpu()) < 1e-5 and _rel(db2.cpu(), D.cpu().sum(0)) < 1e-5
    y = torch.sigmoid(torch.randn(256, 64, device=DEV))
    g = torch.empty(256, 64, device=DEV)
    W = torch.randn(64, 100, device=DEV)
    ops.gemm(X, W, g, M=256, N=64, K=100, aux=y, aux_act=ops.ACT_SIGMOID, tile=ops.TILE_SMALL)
    exp = (X.cpu() @ W.cpu().t()) * y.cpu() * (1 - y.cpu())
    assert _rel(g.cpu(), exp) < 1e-5


def test_gemm_identity_asymmetric():
    M = N = K = 64
    A = torch.eye(M)
    B = torch.arange(N * K, dtype=torch.float32).view(N, K) / 1000.0  # asymmetric
    out = torch.zeros(M, N, device=DEV)
    ops.gemm(A.to(DEV), B.to(DEV), out, M=M, N=N, K=K)
    assert torch.allclose(out.cpu(), B.t(), atol=1e-5)


@pytest.mark.parametrize("act", [0, 1, 2, 3])
def test_gemm_epilogue_bias_act_bf16_out(act):
    torch.manual_seed(1)
    M, N, K = 130, 70, 100
    A = torch.randn(M, K, device=DEV)
    B = torch.randn(N, K, device=DEV)
    bias = torch.randn(N, device=DEV)
    out = torch.empty(M, N, device=DEV, dtype=torch.float32)
    ops.gemm(A, B, out, M=M, N=N, K=K, bias=bias, act=act)
    z = A.cpu() @ B.cpu().t() + bias.cpu()
    exp = [z, torch.relu(z), torch.sigmoid(z), torch.tanh(z)][act]
    assert _rel(out.cpu(), exp) < 1e-5


def test_gemm_split_k_atomic_and_aux():
    torch.manual_seed(2)
    M, N, K = 96, 160, 1000
    A = torch.randn(M, K, device=DEV)
    B = torch.randn(N, K, device=DEV)
    out = torch.zeros(M, N, device=DEV)
    ops.gemm(A, B, out, M=M, N=N, K=K, atomic=True, splits=7)
    assert _rel(out.cpu(), A.cpu() @ B.cpu().t()) < 1e-5
    # activation-gradient prologue: x * sigmoid'(y)
    y = torch.rand(M, N, device=DEV)
    out2 = torch.empty(M, N, device=DEV)
    ops.gemm(A, B, out2, M=M, N=N, K=K, aux=y, aux_act=ops.ACT_SIGMOID)
    exp = (A.cpu() @ B.cpu().t()) * y.cpu() * (1 - y.cpu())
    assert _rel(out2.cpu(), exp) < 1e-5


@pytest.mark.parametrize("tile", [0, 1, 2])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_gemm_split_k_fused_epilogue(tile, dtype):
    """split-K without atomics: last-arriving split sums the partials and runs bias+ReLU;
    run twice so the per-tile arrival counters must have been reset by the kernel."""
    torch.manual_seed(5)
    M, N, K = 200, 300, 1500
    A = torch.randn(M, K).to(DEV, dtype)
    B = torch.randn(N, K).to(DEV, dtype)
    bias = torch.randn(N, device=DEV)
    exp = torch.relu(A.float().cpu() @ B.float().cpu().t() + bias.cpu())
    for _ in range(2):
        out = torch.empty(M, N, device=DEV, dtype=torch.float32)
        ops.gemm(A, B, out, M=M, N=N, K=K, bias=bias, act=ops.ACT_RELU, splits=5, tile=tile)
        assert _rel(out.cpu(), exp) < (2e-2 if dtype == torch.bfloat16 else 1e-5)


def test_gemm_ones_row_bias_column():
    M, N, K = 48, 33, 80
    A = torch.randn(M, K, device=DEV)
    B = torch.randn(N, K, device=DEV)
    out = torch.zeros(M, N, device=DEV)
    ops.gemm(A, B, out, M=M, N=N, K=K, b_ones_row=N - 1)
    exp = A.cpu() @ B.cpu().t()
    exp[:, N - 1] = A.cpu().sum(1)
    assert _rel(out.cpu(), exp) < 1e-5


@pytest.mark.parametrize("dtype,splits", [(torch.float32, 1), (torch.float32, 4), (torch.bfloat16, 1),
                                          (torch.bfloat16, 3)])
def test_gemm_ones_row_bias_row(dtype, splits):
    """a_ones_row: W[in][out] weight gradient X^T . dZ with the bias gradient sum_b dZ[b][:] routed from
    the ones row of A to bias_out - RMAJ operands as the reference models' wgrads use them."""
    Bn, IN, OUT = 200, 100, 70
    X = torch.randn(Bn, IN, device=DEV).to(dtype)
    dZ = torch.randn(Bn, OUT, device=DEV).to(dtype)
    gW = torch.zeros(IN, OUT, device=DEV)
    gb = torch.full((OUT,), 9.0, device=DEV)
    ops.gemm(X, dZ, gW, M=IN + 1, N=OUT, K=Bn, amode=ops.RMAJ, lda=IN, bmode=ops.RMAJ, ldb=OUT,
             a_ones_row=IN, bias_out=gb, splits=splits)
    exp = X.float().cpu().t() @ dZ.float().cpu()
    assert _rel(gW.cpu(), exp) < 1e-5
    assert _rel(gb.cpu(), dZ.float().cpu().sum(0)) < 1e-5


def _geom(B, H, W, C, Cout, KH, KW, stride, pad):
    OH = (H + 2 * pad - KH) // stride + 1
    OW = (W + 2 * pad - KW) // stride + 1
    return dict(B=B, H=H, W=W, C=C, Cout=Cout, OH=OH, OW=OW, KH=KH, KW=KW, stride=stride, pad=pad)


CONV_CASES = [
    _geom(4, 28, 28, 1, 32, 5, 5, 1, 2),     # MNIST conv1
    _geom(4, 14, 14, 32, 64, 5, 5, 1, 2),    # MNIST conv2
    _geom(2, 16, 16, 16, 32, 3, 3, 2, 1),    # ResNet downsample
    _geom(2, 8, 8, 64, 128, 1, 1, 1, 0),     # 1x1
]


@pytest.mark.parametrize("g", CONV_CASES)
@pytest.mark.parametrize("pool", [False, True])
def test_conv_fwd(g, pool):
    if pool and (g["OH"] % 2 or g["OW"] % 2):
        pytest.skip("odd output")
    torch.manual_seed(3)
    x = torch.randn(g["B"], g["H"], g["W"], g["C"]).to(DEV, torch.bfloat16)
    w = (torch.randn(g["Cout"], g["KH"], g["KW"], g["C"]) * 0.2).to(DEV, torch.bfloat16)
    b = torch.randn(g["Cout"], device=DEV)
    OHp, OWp = (g["OH"] // 2, g["OW"] // 2) if pool else (g["OH"], g["OW"])
    y = torch.empty(g["B"], OHp, OWp, g["Cout"], device=DEV, dtype=torch.bfloat16)
    am = torch.empty(g["B"], OHp, OWp, g["Cout"], device=DEV, dtype=torch.uint8) if pool else None
    ops.conv_fwd(x, w, b, y, am, g, pool=pool, act=ops.ACT_RELU)
    yr = torch.empty(y.shape, dtype=torch.float32)
    amr = torch.empty(y.shape, dtype=torch.uint8) if pool else None
    ops.conv_fwd(x.cpu(), w.cpu(), b.cpu(), yr, amr, g, pool=pool, act=ops.ACT_RELU)
    assert _rel(y.cpu(), yr) < 2e-2
    if pool:
        # argmax only matters where the pooled value is > 0 (ReLU ties at 0 are irrelevant)
        pos = yr > 0.05
        agree = (am.cpu()[pos] == amr[pos]).float().mean().item()
        assert agree > 0.97


@pytest.mark.parametrize("g", CONV_CASES[1:])
def test_conv_dgrad(g):
    torch.manual_seed(4)
    dy = torch.randn(g["B"], g["OH"], g["OW"], g["Cout"]).to(DEV, torch.bfloat16)
    w = (torch.randn(g["Cout"], g["KH"], g["KW"], g["C"]) * 0.2)
    wt = w.permute(3, 1, 2, 0).contiguous().to(DEV, torch.bfloat16)  # [C][KH][KW][Cout]
    dx = torch.empty(g["B"], g["H"], g["W"], g["C"], device=DEV, dtype=torch.bfloat16)
    ops.conv_dgrad(dy, wt, dx, g)
    ref = torch.empty(dx.shape)
    ops.conv_dgrad(dy.cpu(), wt.cpu(), ref, g)
    assert _rel(dx.cpu(), ref) < 2e-2


def test_conv_dgrad_unpool():
    g = CONV_CASES[1]
    torch.manual_seed(5)
    dy = torch.randn(g["B"], g["OH"], g["OW"], g["Cout"]).to(DEV, torch.bfloat16)
    wt = (torch.randn(g["C"], g["KH"], g["KW"], g["Cout"]) * 0.2).to(DEV, torch.bfloat16)
    pooled = torch.randn(g["B"], g["H"], g["W"], g["C"]).to(DEV, torch.bfloat16)
    am = torch.randint(0, 4, pooled.shape, dtype=torch.uint8).to(DEV)
    dz = torch.empty(g["B"], 2 * g["H"], 2 * g["W"], g["C"], device=DEV, dtype=torch.bfloat16)
    ops.conv_dgrad(dy, wt, dz, g, pooled=pooled, argmax=am)
    ref = torch.empty(dz.shape)
    ops.conv_dgrad(dy.cpu(), wt.cpu(), ref, g, pooled=pooled.cpu(), argmax=am.cpu())
    assert _rel(dz.cpu(), ref) < 2e-2


@pytest.mark.parametrize("g", CONV_CASES)
def test_conv_wgrad(g):
    torch.manual_seed(6)
    x = torch.randn(g["B"], g["H"], g["W"], g["C"]).to(DEV, torch.bfloat16)
    dz = torch.randn(g["B"], g["OH"], g["OW"], g["Cout"]).to(DEV, torch.bfloat16)
    dw = torch.zeros(g["Cout"], g["KH"], g["KW"], g["C"], device=DEV)
    db = torch.zeros(g["Cout"], device=DEV)
    ops.conv_wgrad(dz, x, dw, db, g, scale=0.5)
    dwr = torch.zeros(dw.shape)
    dbr = torch.zeros(g["Cout"])
    ops.conv_wgrad(dz.cpu(), x.cpu(), dwr, dbr, g, scale=0.5)
    assert _rel(dw.cpu(), dwr) < 1e-2
    assert _rel(db.cpu(), dbr) < 1e-2


def test_conv_dgrad_relu_mask():
    g = CONV_CASES[1]
    torch.manual_seed(12)
    dy = torch.randn(g["B"], g["OH"], g["OW"], g["Cout"]).to(DEV, torch.bfloat16)
    wt = (torch.randn(g["C"], g["KH"], g["KW"], g["Cout"]) * 0.2).to(DEV, torch.bfloat16)
    mask = torch.randn(g["B"], g["H"], g["W"], g["C"]).to(DEV, torch.bfloat16)
    dx = torch.empty(g["B"], g["H"], g["W"], g["C"], device=DEV, dtype=torch.bfloat16)
    ops.conv_dgrad(dy, wt, dx, g, relu_mask=mask)
    ref = torch.empty(dx.shape)
    ops.conv_dgrad(dy.cpu(), wt.cpu(), ref, g, relu_mask=mask.cpu())
    assert _rel(dx.cpu(), ref) < 2e-2
    assert float(dx.cpu()[mask.cpu() <= 0].abs().max()) == 0.0


def test_head_xent():
    torch.manual_seed(7)
    B, K, NC = 300, 1024, 10
    h = torch.relu(torch.randn(B, K)).to(DEV, torch.bfloat16)
    w = (torch.randn(NC, K) * 0.05).to(DEV, torch.bfloat16)
    b = torch.randn(NC, device=DEV)
    labels = torch.randint(0, NC, (B,), dtype=torch.int32, device=DEV)

    def run(dev):
        dz = torch.empty(B, K, device=dev, dtype=torch.bfloat16 if dev == DEV else torch.float32)
        dl = torch.empty(B, 16, device=dev, dtype=torch.bfloat16)
        loss = torch.zeros(1, device=dev)
        corr = torch.zeros(1, dtype=torch.int32, device=dev)
        logits = torch.empty(B, NC, device=dev)
        ops.head_xent(h.to(dev), w.to(dev), b.to(dev), labels.to(dev), dz, dl, loss, corr, logits,
                      scale=1.0 / B, inv_keep=1.25)
        # layer weight/bias grads: split-K wgrad GEMM over the dlogit rows with a ones column
        dw = torch.zeros(NC, K, device=dev)
        db = torch.zeros(NC, device=dev)
        ops.gemm(dl, h.to(dev), dw, M=NC, N=K + 1, K=B, amode=ops.RMAJ, lda=16, bmode=ops.RMAJ, ldb=K, ldc=K,
                 b_ones_row=K, bias_out=db, atomic=True, splits=3, tile=4)
        return [t.cpu() for t in (dz, dl, dw, db, loss, logits, corr)]

    got, exp = run(DEV), run("cpu")
    for gt, ex in zip(got[:6], exp[:6]):
        assert _rel(gt, ex) < 2e-2
    assert float(got[1][:, 10:].abs().max()) == 0.0
    assert abs(int(got[6]) - int(exp[6])) <= 2


@pytest.mark.parametrize("B", [1024, 300, 200])
def test_head_wgrad_matches_fp32(B):
    """Dedicated head weight/bias-gradient kernel vs an fp32 reference of the same product."""
    torch.manual_seed(11)
    K, NC = 1024, 10
    h = torch.relu(torch.randn(B, K)).to(DEV, torch.bfloat16)
    dl = torch.zeros(B, 16, dtype=torch.bfloat16, device=DEV)
    dl[:, :NC] = (torch.randn(B, NC) / B).to(DEV, torch.bfloat16)
    dw = torch.full((NC, K), float("nan"), device=DEV)   # every element must be stored
    db = torch.full((NC,), float("nan"), device=DEV)
    ops.head_wgrad(dl, h, dw, db, NC, scale=0.5)
    ref_w = 0.5 * dl[:, :NC].float().t().cpu() @ h.float().cpu()
    ref_b = 0.5 * dl[:, :NC].float().sum(0).cpu()
    assert _rel(dw.cpu(), ref_w) < 1e-5 and _rel(db.cpu(), ref_b) < 1e-5
    dw2 = torch.empty_like(dw)
    db2 = torch.empty_like(db)
    ops.head_wgrad(dl, h, dw2, db2, NC, scale=0.5)
    assert torch.equal(dw, dw2) and torch.equal(db, db2)   # fixed summation order


@pytest.mark.parametrize("B,grouped", [(1024, True), (1024, False), (301, False)])
def test_head_loss_partials_fold(B, grouped):
    """head_xent's per-workgroup loss / hit partials folded by the head weight gradient's bias
    workgroup == the atomic accumulation; the fold is bitwise reproducible.  (grouped: through a
    gemm_group holding only the head piece - the one-by-one fallback; the fused grouped launch is
    covered by the MNIST CNN step tests' loss checks.)"""
    torch.manual_seed(12)
    K, NC = 1024, 10
    h = torch.relu(torch.randn(B, K)).to(DEV, torch.bfloat16)
    w = (torch.randn(NC, K) * 0.05).to(DEV, torch.bfloat16)
    b = torch.randn(NC, device=DEV)
    labels = torch.randint(0, NC, (B,), dtype=torch.int32, device=DEV)
    dz = torch.empty(B, K, device=DEV, dtype=torch.bfloat16)
    dl = torch.empty(B, 16, device=DEV, dtype=torch.bfloat16)
    dw = torch.empty(NC, K, device=DEV)
    db = torch.empty(NC, device=DEV)
    loss_a = torch.full((1,), 3.0, device=DEV)
    corr_a = torch.full((1,), 5, dtype=torch.int32, device=DEV)
    ops.head_xent(h, w, b, labels, dz, dl, loss_a, corr_a, scale=1.0 / B)
    parts = torch.full((2 * ((B + 3) // 4),), float("nan"), device=DEV)
    outs = []
    for _ in range(2):
        loss = torch.full((1,), 3.0, device=DEV)
        corr = torch.full((1,), 5, dtype=torch.int32, device=DEV)
        ops.head_xent(h, w, b, labels, dz, dl, loss, corr, scale=1.0 / B, parts=parts)
        assert float(loss) == 3.0 and int(corr) == 5   # untouched until the fold
        if grouped:
            with ops.gemm_group(dz):
                ops.head_wgrad(dl, h, dw, db, NC, parts=parts, loss_sum=loss, correct=corr)
        else:
            ops.head_wgrad(dl, h, dw, db, NC, parts=parts, loss_sum=loss, correct=corr)
        outs.append((loss.clone(), corr.clone()))
    assert int(outs[0][1]) == int(corr_a)
    assert abs(float(outs[0][0]) - float(loss_a)) < 1e-4 * abs(float(loss_a))
    assert torch.equal(outs[0][0], outs[1][0])   # fixed summation order


def _plan(n, dev):
    segs = torch.tensor([[0, n, 1, 1, 0, 0]], dtype=torch.int64)
    work = torch.tensor([[0, 0, 0, 0, 0, 0, n]], dtype=torch.int64)
    return ops.opt_pack(segs, work, torch.empty(1, device=dev)), 1, 1


@pytest.mark.parametrize("kind", [0, 1, 2, 3])
def test_optimizers_tf1_math(kind):
    torch.manual_seed(8)
    n = 5000
    p0 = torch.randn(n)
    g = torch.randn(n)
    p = p0.clone().to(DEV)
    s1 = (torch.ones(n) if kind == ops.OPT_RMSPROP else torch.zeros(n)).to(DEV)
    s2 = torch.zeros(n, device=DEV)
    bp = torch.tensor([0.9, 0.999], device=DEV)
    gs = torch.zeros(1, dtype=torch.int32, device=DEV)
    done = torch.zeros(1, dtype=torch.int32, device=DEV)
    blob, ns, nw = _plan(n, DEV)
    lr, b1, b2, eps, mom, rho = 0.01, 0.9, 0.999, 1e-8, 0.5, 0.9
    reps = 3
    for _ in range(reps):
        ops.apply_gradients(kind, p, g.to(DEV), None, 1.0, s1, s2, lr, b1, b2, eps if kind == 2 else 1e-10, mom, rho,
                            bp, gs, 1, done, blob, ns, nw)
    # closed form
    v = p0.clone()
    a1 = torch.ones(n) if kind == 3 else torch.zeros(n)
    a2 = torch.zeros(n)
    b1p, b2p = 0.9, 0.999
    for _ in range(reps):
        if kind == 0:
            v -= lr * g
        elif kind == 1:
            a1 = a1 * mom + g
            v -= lr * a1
        elif kind == 2:
            lr_t = lr * (1 - b2p) ** 0.5 / (1 - b1p)
            a1 = b1 * a1 + (1 - b1) * g
            a2 = b2 * a2 + (1 - b2) * g * g
            v -= lr_t * a1 / (a2.sqrt() + eps)
            b1p *= b1
            b2p *= b2
        else:
            a1 = rho * a1 + (1 - rho) * g * g
            a2 = mom * a2 + lr * g / (a1 + 1e-10).sqrt()
            v -= a2
    assert torch.allclose(p.cpu(), v, atol=1e-5, rtol=1e-5)
    assert int(gs.item()) == reps
    if kind == 2:
        assert abs(bp[0].item() - 0.9 ** (reps + 1)) < 1e-6


def test_grouped_apply_equals_separate_launches():
    """Optimizer.step_all (one grouped launch of the GAN's two Adams) == two separate steps,
    bitwise, including each optimizer's beta powers and the global step."""
    from dtfe.models.gan import GanModel
    from dtfe.optim import Optimizer
    model = GanModel()
    res = []
    for grouped in (False, True):
        prog = model.program(DEV, 32, seed=3)
        torch.manual_seed(5)
        prog.P.grad.copy_(torch.randn(prog.P.total))
        gs = torch.zeros(1, dtype=torch.int32, device=DEV)
        opts = [Optimizer(c, prog.P, var_list=vl, global_step=gs, beta_power_names=bp) for c, vl, bp in model.opt_groups]
        for _ in range(3):
            if grouped:
                Optimizer.step_all(opts, [0, 2])
            else:
                opts[0].step(gs_inc=0)
                opts[1].step(gs_inc=2)
        torch.cuda.synchronize()
        res.append((prog.P.master.cpu(), opts[0].s1.cpu(), opts[1].s2.cpu(), opts[0].beta_pow.cpu(),
                    opts[1].beta_pow.cpu(), int(gs.item())))
    for a, b in zip(*res):
        assert torch.equal(a, b) if torch.is_tensor(a) else a == b
    assert res[1][5] == 6


def test_uniform_fill_fused_copy():
    x = torch.randn(128, 784, device=DEV)
    dst = torch.zeros(256, 784, device=DEV)
    z = torch.empty(128, 100, device=DEV)
    z2 = torch.empty(128, 100, device=DEV)
    ctr = torch.zeros(1, dtype=torch.int64, device=DEV)
    ctr2 = torch.zeros(1, dtype=torch.int64, device=DEV)
    done = torch.zeros(1, dtype=torch.int32, device=DEV)
    done2 = torch.zeros(1, dtype=torch.int32, device=DEV)
    ops.uniform_fill(z, -1.0, 1.0, seed=9, counter=ctr, done=done, copy=(x, dst[:128]))
    ops.uniform_fill(z2, -1.0, 1.0, seed=9, counter=ctr2, done=done2)
    torch.cuda.synchronize()
    assert torch.equal(dst[:128], x) and float(dst[128:].abs().max()) == 0.0
    assert torch.equal(z, z2) and int(ctr.item()) == 1 and float(z.abs().max()) <= 1.0


def test_optimizer_transposed_copies():
    R, T, C = 70, 3, 50
    n = R * T * C
    p = torch.randn(n, device=DEV)
    g = torch.zeros(n, device=DEV)
    w16 = torch.empty(n, device=DEV, dtype=torch.bfloat16)
    wt16 = torch.empty(n, device=DEV, dtype=torch.bfloat16)
    segs = torch.tensor([[0, R, T, C, w16.data_ptr(), wt16.data_ptr()]], dtype=torch.int64)
    work = []
    for t in range(T):
        for r0 in range(0, R, 64):
            for c0 in range(0, C, 64):
                work.append([1, 0, t, r0, c0, 0, 0])
    blob = ops.opt_pack(segs, torch.tensor(work, dtype=torch.int64), p)
    done = torch.zeros(1, dtype=torch.int32, device=DEV)
    ops.apply_gradients(0, p, g, None, 1.0, None, None, 0.1, 0, 0, 0, 0, 0, None, None, 0, done, blob, 1, len(work))
    torch.cuda.synchronize()
    assert torch.equal(w16.cpu(), p.cpu().to(torch.bfloat16))
    exp_t = p.cpu().view(R, T, C).permute(2, 1, 0).reshape(-1).to(torch.bfloat16)
    assert torch.equal(wt16.cpu(), exp_t)


def test_gather_and_noise():
    src = torch.randint(0, 256, (1000, 784), dtype=torch.uint8, device=DEV)
    labels = torch.randint(0, 10, (1000,), dtype=torch.int32, device=DEV)
    idx = torch.randint(0, 1000, (64,), dtype=torch.int32, device=DEV)
    dst = torch.empty(64, 784, device=DEV, dtype=torch.bfloat16)
    ld = torch.empty(64, dtype=torch.int32, device=DEV)
    ops.gather_rows(src, dst, idx, labels, ld)
    exp = src.cpu()[idx.cpu().long()].float() / 255
    assert _rel(dst.cpu(), exp) < 1e-2
    assert torch.equal(ld.cpu(), labels.cpu()[idx.cpu().long()])
    # device sampling: counter advances once per call
    ctr = torch.zeros(1, dtype=torch.int64, device=DEV)
    done = torch.zeros(1, dtype=torch.int32, device=DEV)
    ops.gather_rows(src, dst, None, labels, ld, seed=5, counter=ctr, done=done)
    ops.gather_rows(src, dst, None, labels, ld, seed=5, counter=ctr, done=done)
    assert int(ctr.item()) == 2
    z = torch.empty(128, 100, device=DEV)
    ops.uniform_fill(z, -1.0, 1.0, seed=3, counter=ctr, done=done)
    assert -1.0 <= z.min().item() and z.max().item() < 1.0 and abs(z.mean().item()) < 0.05


def test_gather_long_rows():
    # 224x224x3 images: items of one row spread over many workgroups
    src = torch.randint(0, 256, (20, 224 * 224 * 3), dtype=torch.uint8, device=DEV)
    labels = torch.randint(0, 1000, (20,), dtype=torch.int32, device=DEV)
    idx = torch.tensor([3, 19, 0, 7, 7], dtype=torch.int32, device=DEV)
    dst = torch.empty(5, 224 * 224 * 3, device=DEV, dtype=torch.bfloat16)
    ld = torch.empty(5, dtype=torch.int32, device=DEV)
    ops.gather_rows(src, dst, idx, labels, ld)
    exp = src.cpu()[idx.cpu().long()].float() / 255
    assert _rel(dst.cpu(), exp) < 1e-2
    assert torch.equal(ld.cpu(), labels.cpu()[idx.cpu().long()])


def test_softmax_xent_and_losses():
    torch.manual_seed(9)
    B, NC = 77, 10
    lg = torch.randn(B, NC, device=DEV)
    lab = torch.randint(0, NC, (B,), dtype=torch.int32, device=DEV)
    outs = {}
    for dev in (DEV, "cpu"):
        d = torch.empty(B, NC, device=dev)
        rows = torch.empty(B, device=dev)
        s = torch.zeros(1, device=dev)
        c = torch.zeros(1, dtype=torch.int32, device=dev)
        ops.softmax_xent(lg.to(dev), labels_i=lab.to(dev), scale=1.0 / B, dlogits=d, loss_rows=rows, loss_sum=s,
                         correct=c)
        outs[dev] = [t.cpu() for t in (d, rows, s, c)]
    for a, b in zip(outs[DEV], outs["cpu"]):
        assert _rel(a, b) < 1e-4
    # gan + mse
    pr, pf = torch.rand(128, device=DEV) * 0.9 + 0.05, torch.rand(128, device=DEV) * 0.9 + 0.05
    res = {}
    for dev in (DEV, "cpu"):
        t = [torch.empty(1, device=dev), torch.empty(1, device=dev)] + [torch.empty(128, device=dev) for _ in range(3)]
        ops.gan_loss(pr.to(dev), pf.to(dev), *t)
        res[dev] = [x.cpu() for x in t]
    for a, b in zip(res[DEV], res["cpu"]):
        assert _rel(a, b) < 1e-4
    y, tt = torch.rand(256, 784, device=DEV), torch.rand(256, 784, device=DEV)
    l1, d1 = torch.empty(1, device=DEV), torch.empty_like(y)
    ops.mse_sigmoid(y, tt, l1, d1)
    l2, d2 = torch.empty(1), torch.empty(256, 784)
    ops.mse_sigmoid(y.cpu(), tt.cpu(), l2, d2)
    assert _rel(l1.cpu(), l2) < 1e-4 and _rel(d1.cpu(), d2) < 1e-4


@pytest.mark.parametrize("B", [128, 37])
def test_seq_stage_matches_reference(B):
    """seq_stage (LSTM batch staging in one launch) == the CPU reference: x rows transposed into
    the [T][B][I+H] step rows, h_{-1} zeroed, labels copied, accumulators cleared."""
    T, I, H, NC = 28, 28, 128, 10
    g = torch.Generator().manual_seed(11)
    x = torch.rand(B, T * I, generator=g)
    y = torch.rand(B, NC, generator=g)
    xh_ref = torch.randn(T, B, I + H, generator=g)
    xh = xh_ref.to(DEV)
    y_dst = torch.full((B, NC), 7.0, device=DEV)
    acc_f, acc_i = torch.ones(1, device=DEV), torch.ones(3, dtype=torch.int32, device=DEV)
    ops.seq_stage(x.to(DEV), xh, T, I, y.to(DEV), y_dst, zero=(acc_f, acc_i))
    y_ref, zf, zi = torch.empty(B, NC), torch.ones(1), torch.ones(3, dtype=torch.int32)
    ops.seq_stage(x, xh_ref, T, I, y, y_ref, zero=(zf, zi))
    torch.cuda.synchronize()
    assert torch.equal(xh.cpu(), xh_ref)
    assert torch.equal(y_dst.cpu(), y_ref)
    assert acc_f.item() == 0.0 and int(acc_i.abs().sum().item()) == 0


@pytest.mark.parametrize("M,N,K,splits", [(156, 512, 3584, 32), (156, 512, 3584, 7), (30, 64, 101, 4), (100, 128, 5, 32)])
def test_wgrad_tallk_matches_fp64(M, N, K, splits):
    """Tall-K fp32 weight gradient (LSTM kernel/bias grads) vs a float64 reference, strided rows."""
    g = torch.Generator().manual_seed(M + K)
    lda, ldb = M + 3, N + 8
    A = torch.randn(K, lda, generator=g)
    Bm = torch.randn(K, ldb, generator=g)
    out = torch.full((M, N + 5), 9.0, device=DEV)
    bias = torch.full((N,), 9.0, device=DEV)
    ops.wgrad_tallk(A.to(DEV), lda, Bm.to(DEV), ldb, M, N, K, out, ldc=N + 5, bias=bias, splits=splits, scale=0.5)
    ref = 0.5 * (A[:, :M].double().t() @ Bm[:, :N].double())
    rb = 0.5 * Bm[:, :N].double().sum(0)
    torch.cuda.synchronize()
    o = out.cpu().double()
    assert (o[:, :N] - ref).abs().max().item() <= 1e-4 * (ref.abs().max().item() + 1)
    assert (o[:, N:] == 9.0).all()  # columns past N untouched
    assert (bias.cpu().double() - rb).abs().max().item() <= 1e-4 * (rb.abs().max().item() + 1)




@pytest.mark.parametrize("dtype,tile", [(torch.float32, 0), (torch.bfloat16, 0), (torch.bfloat16, 2)])
def test_splitk_combine_many_splits_deterministic(dtype, tile):
    """Write-through split-K hand-off (gemm_dense.h): 8 split workgroups per tile on a small M x N,
    so every tile's last arriver reads 7 slabs written by workgroups on other XCDs.  Ten launches
    in one process must agree bit for bit, and with the fp64 oracle."""
    torch.manual_seed(3)
    M, N, K = 64, 96, 8 * 512
    A = torch.randn(M, K, device=DEV).to(dtype)
    B = torch.randn(N, K, device=DEV).to(dtype)
    ref = (A.double() @ B.double().t()).float()
    outs = []
    for _ in range(10):
        out = torch.full((M, N), 7.0, device=DEV)
        ops.gemm(A, B, out, M=M, N=N, K=K, splits=8, tile=tile)
        outs.append(out)
    torch.cuda.synchronize()
    for o in outs[1:]:
        assert torch.equal(o, outs[0])
    err = (outs[0] - ref).abs().max().item()
    assert err < 1e-3 * ref.abs().max().item() + 1e-3, err


@pytest.mark.parametrize("g", CONV_CASES + [_geom(2, 14, 14, 6, 16, 3, 3, 2, 1)])
def test_conv_wgrad_fp32(g):
    """conv_f32.hip weight + bias gradient (fp32 tensors route there) vs fp64 autograd: 16-B tap loads
    (C % 4 == 0), per-element loads (C = 1, 6), strides, the bias column."""
    torch.manual_seed(7)
    x = torch.randn(g["B"], g["H"], g["W"], g["C"], device=DEV)
    dz = torch.randn(g["B"], g["OH"], g["OW"], g["Cout"], device=DEV)
    dw = torch.zeros(g["Cout"], g["KH"], g["KW"], g["C"], device=DEV)
    db = torch.zeros(g["Cout"], device=DEV)
    ops.conv_wgrad(dz, x, dw, db, g, scale=0.5)
    xd = x.double().permute(0, 3, 1, 2).requires_grad_(True)
    wd = torch.zeros(g["Cout"], g["C"], g["KH"], g["KW"], dtype=torch.float64, device=DEV, requires_grad=True)
    y = torch.nn.functional.conv2d(xd, wd, stride=g["stride"], padding=g["pad"])
    y.backward(dz.double().permute(0, 3, 1, 2) * 0.5)
    ref_w = wd.grad.permute(0, 2, 3, 1)
    ref_b = 0.5 * dz.double().sum((0, 1, 2))
    assert ((dw.double() - ref_w).abs().max() / ref_w.abs().max()).item() < 1e-5
    assert ((db.double() - ref_b).abs().max() / ref_b.abs().max()).item() < 1e-5


@pytest.mark.parametrize("B,H,K", [(5, 28, 5), (300, 28, 5), (3, 16, 3), (1030, 28, 5)])
def test_conv1_fwd_pool_f32_matches_fp64(B, H, K):
    """The 1-channel fp32 forward (conv1_fwd_pool_f32_kernel: LDS image, packed fp32 FMA, fused bias +
    ReLU + 2x2 max-pool + argmax) vs an fp64 conv2d reference; several images per workgroup
    (B > 1024: the persistent grid), odd batch sizes, 3x3 and 5x5."""
    torch.manual_seed(17)
    g = _geom(B, H, H, 1, 32, K, K, 1, K // 2)
    x = torch.rand(B, H, H, 1, device=DEV)
    w = torch.randn(32, K, K, 1, device=DEV) * 0.2
    b = torch.randn(32, device=DEV) * 0.1
    y = torch.empty(B, H // 2, H // 2, 32, device=DEV)
    am = torch.empty(B, H // 2, H // 2, 32, device=DEV, dtype=torch.uint8)
    ops.conv_fwd(x, w, b, y, am, g, pool=True, act=ops.ACT_RELU)
    z = torch.nn.functional.conv2d(x.double().permute(0, 3, 1, 2), w.double().permute(0, 3, 1, 2), b.double(),
                                   padding=K // 2)
    zz = z.view(B, 32, H // 2, 2, H // 2, 2).permute(0, 2, 4, 1, 3, 5).reshape(B, H // 2, H // 2, 32, 4)
    mx, idx = zz.max(-1)
    assert (y.double() - mx.clamp_min(0)).abs().max().item() < 1e-5
    # argmax: wherever the window's maximum is unambiguous (fp32 ties / near-ties aside)
    top2 = zz.topk(2, -1).values
    clear = (top2[..., 0] - top2[..., 1]) > 1e-5
    assert torch.equal(am.long()[clear], idx[clear])


@pytest.mark.parametrize("B,H,K", [(6, 28, 5), (1024, 28, 5), (7, 16, 3)])
def test_conv1_wgrad_pooled_f32_matches_unpooled_fp64(B, H, K):
    """conv1_wgrad_pooled_f32 (weight + bias gradient from the pooled gradient and its argmax, only the
    argmax pixels, per-workgroup slabs + fixed-order reduce) vs fp64 autograd over the un-pooled
    gradient; accumulates into dw / db (scale), and two launches give identical bits."""
    torch.manual_seed(19)
    g = _geom(B, H, H, 1, 32, K, K, 1, K // 2)
    x = torch.rand(B, H, H, 1, device=DEV)
    dp = torch.randn(B, H // 2, H // 2, 32, device=DEV) * (torch.rand(B, H // 2, H // 2, 32, device=DEV) > 0.3)
    am = torch.randint(0, 4, (B, H // 2, H // 2, 32), device=DEV, dtype=torch.uint8)
    outs = []
    for _ in range(2):
        dw = torch.full((32, K, K, 1), 0.25, device=DEV)
        db = torch.full((32,), -0.5, device=DEV)
        ops.conv1_wgrad_pooled_f32(dp, am, x, dw, db, g, scale=0.5)
        outs.append((dw, db))
    torch.cuda.synchronize()
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    dy = torch.zeros(B, H, H, 32, dtype=torch.float64, device=DEV)
    q = am.long()
    for d in range(4):
        dy[:, d >> 1::2, d & 1::2, :] = torch.where(q == d, dp.double(), torch.zeros_like(dp.double()))
    xd = x.double().permute(0, 3, 1, 2)
    ref_w = torch.nn.grad.conv2d_weight(xd, (32, 1, K, K), dy.permute(0, 3, 1, 2), padding=K // 2)
    ref_w = 0.25 + 0.5 * ref_w.permute(0, 2, 3, 1)
    ref_b = -0.5 + 0.5 * dy.sum((0, 1, 2))
    dw, db = outs[0]
    assert ((dw.double() - ref_w).abs().max() / ref_w.abs().max()).item() < 1e-5
    assert ((db.double() - ref_b).abs().max() / ref_b.abs().max()).item() < 1e-5


@pytest.mark.parametrize("B", [7, 1024])
def test_head_xent_f32_matches_gemm_softmax_chain(B):
    """The fp32 fused head (one launch: logits, softmax-xent sums, dlogits, dZ = dlogits . W * 1/keep *
    ReLU'(h), counter + 1) vs fp64 torch of the same math."""
    torch.manual_seed(23)
    K, NC = 1024, 10
    h = torch.relu(torch.randn(B, K, device=DEV))
    w = torch.randn(NC, K, device=DEV) * 0.05
    b = torch.randn(NC, device=DEV) * 0.1
    lab = torch.randint(0, NC, (B,), device=DEV, dtype=torch.int32)
    dz = torch.empty(B, K, device=DEV)
    dl = torch.empty(B, NC, device=DEV)
    lg = torch.empty(B, NC, device=DEV)
    loss = torch.zeros(1, device=DEV)
    hits = torch.zeros(1, device=DEV, dtype=torch.int32)
    ctr = torch.zeros(1, device=DEV, dtype=torch.int64)
    assert ops.head_xent_f32(h, w, b, lab, dz, dl, loss, hits, logits=lg, scale=1.0 / B, inv_keep=1 / 0.75,
                             step_counter=ctr)
    ref = h.double() @ w.double().t() + b.double()
    p = torch.softmax(ref, 1)
    oh = torch.nn.functional.one_hot(lab.long(), NC).double()
    ref_dl = (p - oh) / B
    ref_dz = (ref_dl @ w.double()) / 0.75 * (h > 0)
    ref_loss = (torch.logsumexp(ref, 1) - ref.gather(1, lab.long()[:, None])[:, 0]).sum()
    assert (lg.double() - ref).abs().max().item() < 1e-4
    assert (dl.double() - ref_dl).abs().max().item() < 1e-6
    assert (dz.double() - ref_dz).abs().max().item() < 1e-6
    assert abs(loss.item() - ref_loss.item()) < 1e-4 * max(1.0, abs(ref_loss.item()))
    assert int(hits.item()) == int((ref.argmax(1) == lab.long()).sum().item())
    assert int(ctr.item()) == 1
