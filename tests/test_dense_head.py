"""The one-launch dense classifier head (ops.dense_head) vs the unfused chain it replaces."""
import pytest
import torch

import dtfe.ops as ops


def _unfused(feat16, w, b, y, B, scale):
    f = feat16.float()
    lg = f @ w.t() + b
    dl = torch.empty_like(lg)
    loss = torch.zeros(1, device=f.device)
    hits = torch.zeros(1, dtype=torch.int32, device=f.device)
    ops.softmax_xent(lg, labels_oh=y, scale=scale, dlogits=dl, loss_sum=loss, correct=hits)
    return lg, loss, hits, dl.t() @ f, dl.sum(0), (dl @ w).bfloat16()


@pytest.mark.gpu
@pytest.mark.parametrize("B,F,NC", [(256, 64, 10), (64, 64, 10), (300, 96, 16)])
def test_dense_head_matches_unfused_gpu(B, F, NC):
    torch.manual_seed(0)
    d = "cuda"
    feat16 = torch.randn(B, F, device=d).bfloat16()
    w, b = torch.randn(NC, F, device=d) * 0.2, torch.randn(NC, device=d) * 0.1
    y = torch.nn.functional.one_hot(torch.randint(0, NC, (B,), device=d), NC).float()
    logits, loss, hits = torch.empty(B, NC, device=d), torch.zeros(1, device=d), torch.zeros(1, dtype=torch.int32, device=d)
    dw, db, dfeat = torch.full((NC, F), 0.5, device=d), torch.full((NC,), 0.25, device=d), torch.empty(B, F, device=d).bfloat16()
    assert ops.dense_head(feat16, w, b, y, logits, loss, hits, dw, db, dfeat, 1.0 / B)
    lg_r, loss_r, hits_r, dw_r, db_r, df_r = _unfused(feat16, w, b, y, B, 1.0 / B)
    assert torch.allclose(logits, lg_r, atol=1e-4, rtol=1e-5)
    assert torch.allclose(loss, loss_r, rtol=1e-5)
    assert int(hits) == int(hits_r)
    assert torch.allclose(dw - 0.5, dw_r, atol=1e-5, rtol=1e-4)   # (+=)
    assert torch.allclose(db - 0.25, db_r, atol=1e-6, rtol=1e-4)
    assert (dfeat.float() - df_r.float()).abs().max() <= 2 * df_r.float().abs().max() * 2 ** -8 + 1e-6


@pytest.mark.gpu
def test_dense_head_declines_what_does_not_fit_gpu():
    """Beyond one workgroup's LDS the launch is declined (False) and the caller runs the unfused chain."""
    d = "cuda"
    B, F, NC = 1024, 64, 10
    z = torch.zeros(NC, F, device=d)
    assert not ops.dense_head(torch.zeros(B, F, device=d).bfloat16(), z, None, torch.zeros(B, NC, device=d), None, None,
                              None, z.clone(), None, torch.empty(B, F, device=d).bfloat16(), 1.0)


def test_dense_head_cpu_oracle():
    torch.manual_seed(1)
    B, F, NC = 8, 16, 4
    feat16 = torch.randn(B, F).bfloat16()
    w, b = torch.randn(NC, F), torch.randn(NC)
    y = torch.nn.functional.one_hot(torch.randint(0, NC, (B,)), NC).float()
    logits, loss, hits = torch.empty(B, NC), torch.zeros(1), torch.zeros(1, dtype=torch.int32)
    dw, db, dfeat = torch.zeros(NC, F), torch.zeros(NC), torch.empty(B, F).bfloat16()
    assert ops.dense_head(feat16, w, b, y, logits, loss, hits, dw, db, dfeat, 1.0 / B)
    lg_r, loss_r, hits_r, dw_r, db_r, df_r = _unfused(feat16, w, b, y, B, 1.0 / B)
    assert torch.allclose(logits, lg_r) and torch.allclose(loss, loss_r) and int(hits) == int(hits_r)
    assert torch.allclose(dw, dw_r) and torch.allclose(db, db_r) and torch.equal(dfeat, df_r)


@pytest.mark.gpu
@pytest.mark.parametrize("B,F,NC", [(128, 128, 10), (40, 64, 10)])
def test_dense_head_fp32_fmajor_store_matches_unfused_gpu(B, F, NC):
    """The LSTM's head form: fp32 features and feature gradient, W / dW laid out [F][NC] (TF Variable
    (in, out)), dW / db stored (not accumulated) - against the unfused fp32 chain."""
    torch.manual_seed(2)
    d = "cuda"
    feat = torch.randn(B, F, device=d)
    w_fnc, b = torch.randn(F, NC, device=d) * 0.2, torch.randn(NC, device=d) * 0.1
    y = torch.nn.functional.one_hot(torch.randint(0, NC, (B,), device=d), NC).float()
    logits, loss, hits = torch.empty(B, NC, device=d), torch.zeros(1, device=d), torch.zeros(1, dtype=torch.int32, device=d)
    dw, db, dfeat = torch.full((F, NC), 9.0, device=d), torch.full((NC,), 9.0, device=d), torch.empty(B, F, device=d)
    assert ops.dense_head(feat, w_fnc, b, y, logits, loss, hits, dw, db, dfeat, 1.0 / B, w_fmajor=True, store=True)
    w = w_fnc.t().contiguous()
    lg_r = feat @ w.t() + b
    dl = torch.empty_like(lg_r)
    loss_r, hits_r = torch.zeros(1, device=d), torch.zeros(1, dtype=torch.int32, device=d)
    ops.softmax_xent(lg_r, labels_oh=y, scale=1.0 / B, dlogits=dl, loss_sum=loss_r, correct=hits_r)
    assert torch.allclose(logits, lg_r, atol=1e-4, rtol=1e-5)
    assert torch.allclose(loss, loss_r, rtol=1e-5) and int(hits) == int(hits_r)
    assert torch.allclose(dw, (dl.t() @ feat).t(), atol=1e-5, rtol=1e-4)
    assert torch.allclose(db, dl.sum(0), atol=1e-6, rtol=1e-4)
    assert torch.allclose(dfeat, dl @ w, atol=1e-6, rtol=1e-4)


@pytest.mark.gpu
def test_dense_head_dlogits_out_without_dfeat_gpu():
    """dl_out (fp32 [B][NC]) instead of dfeat: the dlogits rows the consumer forms dfeat from
    (lstm_seq_bwd(dl=...)) equal softmax_xent's (p - y) * scale."""
    torch.manual_seed(4)
    d, B, F, NC = "cuda", 128, 128, 10
    feat = torch.randn(B, F, device=d)
    w_fnc, b = torch.randn(F, NC, device=d) * 0.2, torch.randn(NC, device=d) * 0.1
    y = torch.nn.functional.one_hot(torch.randint(0, NC, (B,), device=d), NC).float()
    dw, db, dl = torch.empty(F, NC, device=d), torch.empty(NC, device=d), torch.empty(B, NC, device=d)
    assert ops.dense_head(feat, w_fnc, b, y, None, None, None, dw, db, None, 1.0 / B, w_fmajor=True, store=True,
                          dl_out=dl)
    lg = feat @ w_fnc + b
    ref = torch.empty_like(lg)
    ops.softmax_xent(lg, labels_oh=y, scale=1.0 / B, dlogits=ref)
    assert torch.allclose(dl, ref, atol=1e-6, rtol=1e-4)
