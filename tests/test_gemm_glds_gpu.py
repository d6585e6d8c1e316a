"""global_load_lds dense GEMM tiles (csrc/kernels/gemm_glds.h) against an fp32 PyTorch oracle:
every operand layout (KMAJ / RMAJ), every tile, split-K with the fused last-arriver epilogue,
the bias/ReLU/dropout epilogue, the act'(aux) epilogue, and the ones-tile bias column of a
weight-gradient GEMM - on the MNIST-CNN fc1 shapes and asymmetric small ones."""
import pytest
import torch

from dtfe import ops

pytestmark = pytest.mark.gpu
bf = torch.bfloat16


def _mat(t, mode, rows, K):
    """logical [rows, K] of an operand stored KMAJ ([rows][K]) or RMAJ ([K][rows])"""
    return t.float() if mode == ops.KMAJ else t.float().t()


@pytest.mark.parametrize("tile", [5, 6, 7, 8, 9, 12, 14, 15, 16, 17, 18, 19, 20, 21])
@pytest.mark.parametrize("modes", [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize("splits", [1, 3])
def test_glds_gemm_layouts(tile, modes, splits):
    am, bm = modes
    M, N, K = 256, 384, 640
    g = torch.Generator(device="cuda").manual_seed(tile * 10 + am * 2 + bm)
    A = (torch.randn(M, K, device="cuda", generator=g) if am == ops.KMAJ else
         torch.randn(K, M, device="cuda", generator=g)).to(bf)
    B = (torch.randn(N, K, device="cuda", generator=g) if bm == ops.KMAJ else
         torch.randn(K, N, device="cuda", generator=g)).to(bf)
    # asymmetric: make row i of A carry a ramp so a transposed store cannot pass
    out = torch.empty(M, N, device="cuda", dtype=torch.float32)
    ops.gemm(A, B, out, M=M, N=N, K=K, amode=am, bmode=bm, tile=tile, splits=splits)
    ref = _mat(A, am, M, K) @ _mat(B, bm, N, K).t()
    err = (out - ref).abs().max().item() / ref.abs().max().item()
    assert err < 1e-5, err


@pytest.mark.parametrize("tile,splits", [(5, 4), (6, 2), (8, 1), (19, 1), (20, 2), (21, 1)])
def test_glds_fc1_forward_epilogue(tile, splits):
    """fc1 forward: H = dropout(relu(P2 . W1^T + b)) at B=1024, K=3136."""
    B_, K1, FC = 1024, 3136, 1024
    g = torch.Generator(device="cuda").manual_seed(1)
    p2 = torch.rand(B_, K1, device="cuda", generator=g).to(bf)
    w1 = (torch.randn(FC, K1, device="cuda", generator=g) * 0.02).to(bf)
    bias = torch.randn(FC, device="cuda", generator=g) * 0.1
    ctr = torch.tensor([5], dtype=torch.int64, device="cuda")
    h = torch.empty(B_, FC, device="cuda", dtype=bf)
    h_ref = torch.empty_like(h)
    kw = dict(M=B_, N=FC, K=K1, bias=bias, act=ops.ACT_RELU, keep=0.75, seed=9, counter=ctr)
    ops.gemm(p2, w1, h, tile=tile, splits=splits, **kw)
    ops.gemm(p2, w1, h_ref, tile=0, splits=1, **kw)   # register-staged engine: same epilogue + mask
    z = torch.relu(p2.float() @ w1.float().t() + bias)
    keep_mask = h_ref != 0
    # the same hash-RNG dropout mask (up to values that round to 0 in one of the two)
    assert ((h != 0) == keep_mask).float().mean().item() > 0.999
    ref = torch.where(keep_mask, z / 0.75, torch.zeros_like(z))
    err = (h.float() - ref).abs().max().item() / ref.abs().max().item()
    assert err < 1e-2, err


def test_glds_fc1_dgrad_and_wgrad():
    """fc1 data gradient (B operand RMAJ, act'(aux) epilogue) and weight gradient (both RMAJ,
    fp32 out, bias gradient through the ones tile)."""
    B_, K1, FC = 1024, 3136, 1024
    g = torch.Generator(device="cuda").manual_seed(2)
    dz = torch.randn(B_, FC, device="cuda", generator=g).to(bf)
    w1 = (torch.randn(FC, K1, device="cuda", generator=g) * 0.02).to(bf)
    p2 = torch.relu(torch.randn(B_, K1, device="cuda", generator=g)).to(bf)
    dp2 = torch.empty(B_, K1, device="cuda", dtype=bf)
    ops.gemm(dz, w1, dp2, M=B_, N=K1, K=FC, bmode=ops.RMAJ, ldb=K1, aux=p2, aux_act=ops.ACT_RELU, tile=8)
    ref = (dz.float() @ w1.float()) * (p2.float() > 0)
    err = (dp2.float() - ref).abs().max().item() / ref.abs().max().item()
    assert err < 1e-2, err
    gw = torch.full((FC, K1), 7.0, device="cuda")
    gb = torch.full((FC,), 7.0, device="cuda")
    dp2b = torch.empty_like(dp2)
    ops.gemm(dz, w1, dp2b, M=B_, N=K1, K=FC, bmode=ops.RMAJ, ldb=K1, aux=p2, aux_act=ops.ACT_RELU, tile=ops.FC_TILE)
    err = (dp2b.float() - ref).abs().max().item() / ref.abs().max().item()
    assert err < 1e-2, err
    for tile, splits in ((8, 1), (8, 2), (6, 1), (12, 1), (19, 1), (20, 1), (22, 1), (22, 2)):
        if not ops.glds_ok(dz, p2, FC, K1 + 1, B_, tile, FC, K1, b_ones_row=K1, bmode=ops.RMAJ):
            continue
        ops.gemm(dz, p2, gw, M=FC, N=K1 + 1, K=B_, amode=ops.RMAJ, lda=FC, bmode=ops.RMAJ, ldb=K1, ldc=K1,
                 b_ones_row=K1, bias_out=gb, tile=tile, splits=splits)
        ref_w = dz.float().t() @ p2.float()
        ref_b = dz.float().sum(0)
        assert (gw - ref_w).abs().max().item() < 1e-4 * ref_w.abs().max().item() + 1e-3, (tile, splits)
        assert (gb - ref_b).abs().max().item() < 1e-4 * ref_b.abs().max().item() + 1e-3, (tile, splits)


@pytest.mark.parametrize("modes", [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize("N", [384, 200, 3136])
@pytest.mark.parametrize("splits", [1, 3])
def test_fc_tile22_layouts(modes, N, splits):
    """tile 22 (8-wave 256x128, gemm_fc.hip): every layout, a partial last n-tile (RMAJ B: sources
    clamped inside the row, outputs past N never stored), split-K with the last-arriver epilogue."""
    tile = ops.FC_TILE
    am, bm = modes
    M, K = 512, 640
    g = torch.Generator(device="cuda").manual_seed(N + am * 2 + bm)
    A = (torch.randn(M, K, device="cuda", generator=g) if am == ops.KMAJ else
         torch.randn(K, M, device="cuda", generator=g)).to(bf)
    B = (torch.randn(N, K, device="cuda", generator=g) if bm == ops.KMAJ else
         torch.randn(K, N, device="cuda", generator=g)).to(bf)
    eligible = ops.glds_ok(A, B, M, N, K, tile, K if am == 0 else M, K if bm == 0 else N, bmode=bm)
    assert eligible == (bm == ops.RMAJ or N % 128 == 0)
    if not eligible:
        return
    out = torch.full((M, N + 8), 123.0, device="cuda")
    ops.gemm(A, B, out, M=M, N=N, K=K, amode=am, bmode=bm, ldc=N + 8, tile=tile, splits=splits)
    ref = _mat(A, am, M, K) @ _mat(B, bm, N, K).t()
    err = (out[:, :N] - ref).abs().max().item() / ref.abs().max().item()
    assert err < 1e-5, err
    assert (out[:, N:] == 123.0).all()  # nothing stored past N


@pytest.mark.parametrize("tile", [12, 22])
def test_gemm_group_matches_separate_launches(tile):
    """ops.gemm_group: the head weight gradient + fc1 data gradient + fc1 weight gradient recorded
    and launched as ONE grid give bitwise the results of the separate launches (tile 22: the group's
    per-wave head body sums in another order than head_wgrad's kernel - head compared to 1e-5)."""
    B_, K1, FC, NC = 1024, 3136, 1024, 10
    g = torch.Generator(device="cuda").manual_seed(3)
    dz = torch.randn(B_, FC, device="cuda", generator=g).to(bf)
    w1 = (torch.randn(FC, K1, device="cuda", generator=g) * 0.02).to(bf)
    p2 = torch.relu(torch.randn(B_, K1, device="cuda", generator=g)).to(bf)
    h = torch.relu(torch.randn(B_, FC, device="cuda", generator=g)).to(bf)
    dl = torch.zeros(B_, 16, device="cuda", dtype=bf)
    dl[:, :NC] = (torch.randn(B_, NC, device="cuda", generator=g) / B_).to(bf)

    def run(grouped):
        dp2 = torch.full((B_, K1), float("nan"), device="cuda").to(bf)
        gw = torch.full((FC, K1), float("nan"), device="cuda")
        gb = torch.full((FC,), float("nan"), device="cuda")
        hw = torch.full((NC, FC), float("nan"), device="cuda")
        hb = torch.full((NC,), float("nan"), device="cuda")
        ctx = ops.gemm_group(dz) if grouped else __import__("contextlib").nullcontext()
        with ctx:
            ops.head_wgrad(dl, h, hw, hb, NC)
            ops.gemm(dz, w1, dp2, M=B_, N=K1, K=FC, bmode=ops.RMAJ, ldb=K1, aux=p2, aux_act=ops.ACT_RELU, tile=tile)
            ops.gemm(dz, p2, gw, M=FC, N=K1 + 1, K=B_, amode=ops.RMAJ, lda=FC, bmode=ops.RMAJ, ldb=K1, ldc=K1,
                     b_ones_row=K1, bias_out=gb, tile=tile)
        torch.cuda.synchronize()
        return dp2, gw, gb, hw, hb

    sep, grp = run(False), run(True)
    for i, (a, b) in enumerate(zip(sep, grp)):
        assert not torch.isnan(b.float()).any()
        if tile == 22 and i >= 3:
            assert (a - b).abs().max().item() <= 1e-5 * a.abs().max().item() + 1e-7, i
        else:
            assert torch.equal(a, b), i
    hw_ref = dl[:, :NC].float().t() @ h.float()
    assert (grp[3] - hw_ref).abs().max().item() < 1e-4 * hw_ref.abs().max().item() + 1e-6
    ref = (dz.float() @ w1.float()) * (p2.float() > 0)
    assert (grp[0].float() - ref).abs().max().item() < 1e-2 * ref.abs().max().item()
