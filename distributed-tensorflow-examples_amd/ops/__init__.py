"""Op layer: thin wrappers over ``torch.ops.dtfe`` (gfx950 HIP kernels).

Every op writes into caller-provided tensors (no allocation inside a step, so
steps are hipGraph-capturable).  GPU tensors always go to the HIP kernels -
if the native library is missing that is an error, never a silent fallback.
CPU tensors take a plain-PyTorch reference path: it exists for the CPU/gloo
plumbing configuration (BASELINE.json config 1), for CPU tests of the
distributed machinery, and as the fp32 oracle the kernel tests compare to.
"""
from __future__ import annotations

import contextlib
import math
import os

import numpy as np
import torch

from ._lib import (ACT_CODES, ACT_NONE, ACT_RELU, ACT_SIGMOID, ACT_TANH, KMAJ, OPT_ADAM, OPT_MOMENTUM,
                   OPT_RMSPROP, OPT_SGD, RMAJ, available, load, require)

__all__ = [
    "gemm", "linear_fwd", "conv_fwd", "conv_dgrad", "conv_wgrad", "head_xent", "apply_gradients", "opt_pack",
    "gather_rows", "uniform_fill", "cast_", "softmax_xent", "gan_loss", "mse_sigmoid", "colsum", "act_grad",
    "bias_act", "ACT_NONE", "ACT_RELU", "ACT_SIGMOID", "ACT_TANH", "ACT_CODES", "KMAJ", "RMAJ", "OPT_SGD",
    "OPT_MOMENTUM", "OPT_ADAM", "OPT_RMSPROP", "available", "load", "require", "pick_tile", "split_workspace",
    "TILE_DIMS", "FC_TILE", "TILE_SMALL", "GEMM_KTILE", "GLDS_TILES", "glds_ok", "ones_page", "bn_stats", "bn_apply", "bn_bwd_stats",
    "bn_bwd_apply", "relu_bits", "shortcut_grad_add",
    "gap_fwd", "gap_bwd", "gemm_group", "seq_stage", "wgrad_tallk", "tallk_ws_floats", "maxpool3_fwd", "maxpool3_bwd", "bn_relu_pool3", "pool3_bn_bwd", "imgconv", "imgwgrad", "hash_uniform",
    "imgconv_shortcut", "dense_head", "wgrad_flush", "wgrad_pending", "wgrad_discard", "conv1_wgrad_pooled_f32",
    "head_xent_f32", "gan_disc_head", "gan_head_ws_floats", "apply_wait_next", "epoch_signal",
]

_TILES = [(1, 128, 128), (2, 128, 64), (3, 64, 128), (0, 64, 64)]
TILE_DIMS = {0: (64, 64), 1: (128, 128), 2: (128, 64), 3: (64, 128), 4: (32, 32),
             # global_load_lds kernel family (csrc/kernels/gemm_glds.h): bf16, K % 64 == 0, whole tiles
             5: (128, 128), 6: (128, 64), 7: (64, 128), 8: (64, 64),      # 3 k-tiles in flight
             9: (128, 128), 10: (128, 64), 11: (64, 128), 12: (64, 64),   # 2 stages (more WGs per CU)
             13: (16, 16),   # exact-fp32 small-layer kernel (gemm_small.hip): no split-K, in-WG K split
             14: (64, 64), 15: (64, 64), 16: (64, 64),  # 4 / 6 / 8 stages (long-K grids, ~1 WG per CU)
             17: (128, 64), 18: (128, 64),              # 4 / 6 stages
             19: (64, 64), 20: (64, 64), 21: (64, 64),  # 2 / 4 / 2 in-workgroup k-groups (3 / 2 / 4 stages)
             22: (256, 128)}  # 8-wave fc tile (gemm_fc.hip): M % 256, N any (clamped last tile), 3 stages
FC_TILE = 22
GLDS_TILES = (5, 6, 7, 8, 9, 10, 11, 12, 14, 15, 16, 17, 18, 19, 20, 21, 22)
TILE_SMALL = 13
_ONES = {}


def ones_page(device):
    """1 KB of bf16 ones (the bias column of a glds weight-gradient GEMM reads it)."""
    key = torch.device(device)
    t = _ONES.get(key)
    if t is None:
        t = _ONES[key] = torch.ones(512, dtype=torch.bfloat16, device=key)
    return t


def glds_ok(A, B, M, N, K, tile, lda, ldb, b_ones_row=-1, a_ones_row=-1, bmode=KMAJ):
    """Host mirror of gemm_glds_eligible: can the global_load_lds tile `tile` run this GEMM?"""
    bm, bn = TILE_DIMS[tile]
    if A.dtype != torch.bfloat16 or B.dtype != torch.bfloat16 or a_ones_row >= 0 or K % 64 or M % bm:
        return False
    if lda % 8 or ldb % 8 or A.data_ptr() % 16 or B.data_ptr() % 16:
        return False
    if tile == FC_TILE:  # mirror of gemm_fc_eligible (csrc/kernels/gemm_fc.hip)
        valid = b_ones_row if b_ones_row >= 0 else N
        if b_ones_row >= 0 and (b_ones_row != N - 1 or b_ones_row % 8):
            return False
        return valid >= 8 and valid % 8 == 0 and (bmode == RMAJ or (N % bn == 0 and b_ones_row < 0))
    if b_ones_row >= 0:
        return b_ones_row == N - 1 and b_ones_row % bn == 0
    return N % bn == 0
GEMM_KTILE = 64  # k-tile depth of the dense GEMM kernels (split-K chunks are multiples of it)
_WS = {}
# Every workspace ever handed out stays alive: a hipGraph captured with an older (smaller)
# buffer keeps its device pointers, and the caching allocator must never recycle that memory.
_WS_RETIRED = []


def split_workspace(device, splits, M, N, tile, private=False):
    """(ws, tile_ctr) for a split-K GEMM with a fused epilogue: fp32 partial tiles
    [splits][tiles][BM*BN] + per-tile arrival counters (zeroed once; the kernel
    resets them).  Cached per device and grown on demand - callers that run
    split-K GEMMs concurrently on several streams must pass their own
    (``private=True``: a fresh pair, not the shared cache)."""
    bm, bn = TILE_DIMS[tile]
    ntiles = math.ceil(M / bm) * math.ceil(N / bn)
    need = splits * ntiles * bm * bn
    if private:
        key = torch.device(device)
        return (torch.empty(need, device=key, dtype=torch.float32),
                torch.zeros(ntiles, device=key, dtype=torch.int32))
    key = torch.device(device)
    ws, ctr = _WS.get(key, (None, None))
    if ws is None or ws.numel() < need or ctr.numel() < ntiles:
        if ws is not None:
            _WS_RETIRED.append((ws, ctr))
        ws = torch.empty(max(need, 0 if ws is None else ws.numel()), device=key, dtype=torch.float32)
        ctr = torch.zeros(max(ntiles, 0 if ctr is None else ctr.numel()), device=key, dtype=torch.int32)
        _WS[key] = (ws, ctr)
    return ws, ctr


def auto_splits(M: int, N: int, K: int, tile: int) -> int:
    """Split-K factor for an under-filled GEMM (few output tiles, long K: the small dense layers
    of the reference models, a weight gradient reducing over T*B rows) so the grid reaches
    ~256 workgroups; the last-arriving split runs the fused epilogue (deterministic order).
    Uses the shared per-device workspace: GEMMs issued concurrently on several streams must not
    rely on it (pass splits / workspace explicitly)."""
    if tile == TILE_SMALL:
        return 1
    bm, bn = TILE_DIMS[tile]
    tiles = math.ceil(M / bm) * math.ceil(N / bn)
    if tiles >= 128 or K < 4 * GEMM_KTILE:
        return 1
    return max(1, min(math.ceil(256 / tiles), K // (2 * GEMM_KTILE), 16))


def small_f32_ok(M: int, N: int, K: int) -> bool:
    """The small-layer fp32 kernel wins where the output has at most ~1M elements (<= 4096
    16x16 tiles) and K is short enough for register-direct operands (reference GAN /
    autoencoder layers: 1.7-10 us -> ~2-3 us each); DTFE_GEMM_SMALL=0 disables it."""
    return _SMALL_ON and math.ceil(M / 16) * math.ceil(N / 16) <= 4096 and K <= 2048


_SMALL_ON = os.environ.get("DTFE_GEMM_SMALL", "1") != "0"


def pick_tile(M: int, N: int) -> int:
    """Largest MFMA tile that still yields >= one workgroup per CU (256 CUs)."""
    if M <= 32 and N <= 32:
        return 4
    for tid, bm, bn in _TILES:
        if math.ceil(M / bm) * math.ceil(N / bn) >= 256:
            return tid
    # small outputs: 32x32 tiles quadruple the workgroups of 64x64 (split-K adds more if K allows)
    return 4 if math.ceil(M / 64) * math.ceil(N / 64) < 64 else 0


# --------------------------------------------------------------- references
def hash_uniform(seed, idx):
    """Host mirror of the kernels' counter-based RNG (common.h hash_u32/hash_uniform):
    splitmix-style 64-bit mix of (seed, element index) -> uniform [0, 1) with 24 bits."""
    with np.errstate(over="ignore"):
        z = (np.uint64(seed) * np.uint64(0x9E3779B97F4A7C15) + np.asarray(idx, dtype=np.uint64)
             * np.uint64(0xD1B54A32D192ED03) + np.uint64(0x632BE59BD9B4E019))
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z ^= z >> np.uint64(31)
    return ((z & np.uint64(0xFFFFFFFF)) >> np.uint64(8)).astype(np.float32) * np.float32(1.0 / 16777216.0)


def _act_ref(x, act):
    if act == ACT_RELU:
        return torch.relu(x)
    if act == ACT_SIGMOID:
        return torch.sigmoid(x)
    if act == ACT_TANH:
        return torch.tanh(x)
    return x


def _act_grad_from_out_ref(y, act):
    if act == ACT_RELU:
        return (y > 0).to(y.dtype)
    if act == ACT_SIGMOID:
        return y * (1 - y)
    if act == ACT_TANH:
        return 1 - y * y
    return torch.ones_like(y)


def _mat(t, mode, rows, K, ld):
    """Logical [rows, K] fp32 view of an operand given its mode/leading dim."""
    flat = t.reshape(-1).float()
    if mode == KMAJ:
        idx = torch.arange(rows).unsqueeze(1) * ld + torch.arange(K).unsqueeze(0)
    else:
        idx = torch.arange(K).unsqueeze(0) * ld + torch.arange(rows).unsqueeze(1)
    return flat[idx]


# --------------------------------------------------------------------- GEMM
def gemm(A, B, out, *, M, N, K, amode=KMAJ, lda=None, bmode=KMAJ, ldb=None, ldc=None, bias=None, bias_axis=0,
         act=ACT_NONE, alpha=1.0, beta=0.0, atomic=False, splits=1, tile=None, aux=None, ld_aux=None, aux_act=0,
         b_ones_row=-1, keep=1.0, seed=0, counter=None, pooled=None, argmax=None, PH=0, PW=0, PC=0, out2=None,
         ldc2=0, out2_trans=False, bias_out=None, workspace=None, a_ones_row=-1):
    """out[M,N] = epilogue( A(m,k) . B(n,k) ).

    A(m,k) = A[m*lda+k] (KMAJ) or A[k*lda+m] (RMAJ); likewise B(n,k).
    Epilogue order: alpha*acc, +bias, act, dropout(keep), *act'(aux), [unpool | +beta*out], store.
    b_ones_row >= 0 makes B row n=b_ones_row all ones; with bias_out that output
    column goes to bias_out[m] (a weight-gradient GEMM producing the bias gradient).
    a_ones_row = M-1 is the transpose: A's last row reads as ones and output row M-1 goes to
    bias_out[n] (W[in][out] weight gradients: the bias gradient without a column-sum launch).
    splits > 1 without atomic: split-K whose last-arriving split runs the fused
    epilogue (workspace = (ws, tile_ctr), default: a per-device cached one).
    """
    if lda is None:
        lda = K if amode == KMAJ else M
    if ldb is None:
        ldb = K if bmode == KMAJ else N
    if ldc is None:
        ldc = N
    if ld_aux is None:
        ld_aux = ldc
    if out.is_cuda:
        if tile is None and A.dtype == torch.float32 and pooled is None and splits == 1 and \
                small_f32_ok(M, N, K):
            tile = TILE_SMALL
        if tile is None:
            tile = pick_tile(M, N)
            if splits == 1 and not atomic and workspace is None:
                splits = auto_splits(M, N, K, tile)
        ws = ctr = None
        if splits > 1 and not atomic:
            ws, ctr = workspace if workspace is not None else split_workspace(out.device, splits, M, N, tile)
        require().gemm(A, amode, lda, B, bmode, ldb, M, N, K, out, ldc, bias, bias_axis, act, alpha, beta, atomic,
                       splits, tile, aux, ld_aux, aux_act, b_ones_row, keep, seed, counter, pooled, argmax, PH, PW,
                       PC, out2, ldc2, out2_trans, bias_out, ws, ctr, a_ones_row,
                       ones_page(out.device) if tile in GLDS_TILES else None)
        return out
    # CPU reference
    if a_ones_row >= 0:
        assert a_ones_row == M - 1, "CPU reference: a_ones_row must be the last row"
        a = torch.cat([_mat(A, amode, M - 1, K, lda), torch.ones(1, K)], 0)
    else:
        a = _mat(A, amode, M, K, lda)
    if b_ones_row >= 0:
        b = _mat(B, bmode, b_ones_row, K, ldb) if b_ones_row > 0 else torch.zeros(0, K)
        b = torch.cat([b, torch.ones(1, K), _mat_tail(B, bmode, b_ones_row + 1, N, K, ldb)], 0)
    else:
        b = _mat(B, bmode, N, K, ldb)
    acc = a @ b.t()
    if bias_out is not None and a_ones_row >= 0:
        if atomic:
            bias_out += alpha * acc[a_ones_row]
        else:
            bias_out.copy_(alpha * acc[a_ones_row])
        acc = acc[:a_ones_row]
        M = a_ones_row
    elif bias_out is not None:
        if atomic:
            bias_out += alpha * acc[:, b_ones_row]
        else:
            bias_out.copy_(alpha * acc[:, b_ones_row])
        keep_cols = [c for c in range(N) if c != b_ones_row]
        acc = acc[:, keep_cols]
        N = len(keep_cols)
    oflat = out.view(-1)
    oidx = torch.arange(M).unsqueeze(1) * ldc + torch.arange(N).unsqueeze(0)
    if atomic:
        oflat[oidx] += (alpha * acc).to(out.dtype)
        return out
    x = alpha * acc
    if bias is not None:
        x = x + (bias.float().view(1, -1) if bias_axis == 0 else bias.float().view(-1, 1))
    x = _act_ref(x, act)
    if keep < 1.0:
        step = int(counter.reshape(-1)[0].item()) if counter is not None else 0
        oidx0 = torch.arange(M).unsqueeze(1) * ldc + torch.arange(N).unsqueeze(0)
        u = hash_uniform(seed, oidx0.reshape(-1).numpy().astype(np.uint64) + np.uint64(step * M * N))
        x = torch.where(torch.from_numpy(u).reshape(M, N) < keep, x / keep, torch.zeros_like(x))
    if aux is not None:
        aidx = torch.arange(M).unsqueeze(1) * ld_aux + torch.arange(N).unsqueeze(0)
        x = x * _act_grad_from_out_ref(aux.reshape(-1).float()[aidx], aux_act)
    if pooled is not None:
        _unpool_ref(x.reshape(-1), pooled, argmax, PH, PW, PC, out)
        return out
    if beta != 0.0:
        x = x + beta * oflat[oidx].float()
    oflat[oidx] = x.to(out.dtype)
    if out2 is not None:
        o2 = out2.view(-1)
        idx2 = (torch.arange(N).unsqueeze(0) * ldc2 + torch.arange(M).unsqueeze(1)) if out2_trans else \
            (torch.arange(M).unsqueeze(1) * ldc2 + torch.arange(N).unsqueeze(0))
        o2[idx2] = x.to(out2.dtype)
    return out


def _mat_tail(t, mode, r0, rows, K, ld):
    """Rows r0..rows-1 of the logical [rows, K] operand (those that exist in memory)."""
    if r0 >= rows:
        return torch.zeros(0, K)
    flat = t.reshape(-1).float()
    r = torch.arange(r0, rows)
    if mode == KMAJ:
        idx = r.unsqueeze(1) * ld + torch.arange(K).unsqueeze(0)
    else:
        idx = torch.arange(K).unsqueeze(0) * ld + r.unsqueeze(1)
    return flat[idx]


def _unpool_ref(g, pooled, argmax, PH, PW, C, dz):
    """Route pooled-grad g (flat [B*PH*PW*C]) to argmax positions, ReLU-masked by pooled>0."""
    Bn = g.numel() // (PH * PW * C)
    g = g.view(Bn, PH, PW, C) * (pooled.view(Bn, PH, PW, C).float() > 0)
    am = argmax.view(Bn, PH, PW, C).long()
    full = torch.zeros(Bn, PH, 2, PW, 2, C)
    for q in range(4):
        full[:, :, q >> 1, :, q & 1, :] = torch.where(am == q, g, torch.zeros_like(g))
    dz.view(-1)[:] = full.reshape(-1).to(dz.dtype)


def linear_fwd(x, w_kn, b, out, act=ACT_NONE):
    """TF-layout dense layer: out = act(x[M,K] . W[K,N] + b)."""
    M, K = x.shape[0], x.shape[-1]
    N = w_kn.shape[1]
    return gemm(x, w_kn, out, M=M, N=N, K=K, amode=KMAJ, bmode=RMAJ, ldb=N, bias=b, act=act)


# -------------------------------------------------------------------- conv
def _conv_geom_args(g):
    return (g["B"], g["H"], g["W"], g["C"], g["Cout"], g["OH"], g["OW"], g["KH"], g["KW"], g["stride"], g["pad"])


def conv_fwd(x, w, bias, y, argmax, g, pool=False, act=ACT_RELU, stats=None):
    """NHWC conv (+bias, act, optional fused 2x2 max-pool writing argmax).  ``stats`` (f32 [2][Cout],
    zeroed): also accumulate the BatchNorm statistics of y exactly as ``bn_stats`` does (the
    implicit-GEMM path computes them from its epilogue tiles: no separate pass over y)."""
    if y.is_cuda:
        require().conv_fwd(x, w, bias, y, argmax, *_conv_geom_args(g), pool, act, stats)
        return y
    if stats is not None:
        conv_fwd(x, w, bias, y, argmax, g, pool, act)
        bn_stats(y, stats)
        return y
    xt = x.float().view(g["B"], g["H"], g["W"], g["C"]).permute(0, 3, 1, 2)
    wt = w.float().view(g["Cout"], g["KH"], g["KW"], g["C"]).permute(0, 3, 1, 2)
    z = torch.nn.functional.conv2d(xt, wt, bias.float() if bias is not None else None, stride=g["stride"],
                                   padding=g["pad"])
    z = _act_ref(z, act)
    if pool:
        p, idx = _pool_ref(z)
        y.view(-1)[:] = p.permute(0, 2, 3, 1).reshape(-1).to(y.dtype)
        if argmax is not None:
            argmax.view(-1)[:] = idx.permute(0, 2, 3, 1).reshape(-1).to(argmax.dtype)
    else:
        y.view(-1)[:] = z.permute(0, 2, 3, 1).reshape(-1).to(y.dtype)
    return y


def _pool_ref(z):
    """2x2/2 max pool of NCHW z; returns (pooled, argmax in 0..3 = dy*2+dx, first max wins)."""
    Bn, C, H, W = z.shape
    win = z.view(Bn, C, H // 2, 2, W // 2, 2).permute(0, 1, 2, 4, 3, 5).reshape(Bn, C, H // 2, W // 2, 4)
    p, idx = win.max(dim=-1)
    # torch.max returns the first maximal index on ties
    return p, idx


def _unpooled_nhwc(pooled, argmax, B, H, W, C):
    """Full-resolution NHWC tensor holding pooled[w] at argmax position of each 2x2 window."""
    out = torch.zeros(B * H * W * C)
    _unpool_ref(pooled.reshape(-1).float(), torch.ones(B, H // 2, W // 2, C), argmax, H // 2, W // 2, C, out)
    return out.view(B, H, W, C)


def _bn_src_ref(src, bn_src, eps, momentum, save):
    """CPU oracle of a BN + ReLU formed on a conv's source (bn_src = [stats, gamma, beta, mean,
    invstd, moving_mean, moving_var]): bn_apply's output."""
    st, g, b, m, i, mm, mv = bn_src
    h = torch.empty_like(src)
    kw = dict(mean=m, invstd=i, moving_mean=mm, moving_var=mv) if save else {}
    bn_apply(src, st, g, b, h, eps=eps, momentum=momentum, act=ACT_RELU, **kw)
    return h


def imgconv(w, y, *, B, SH, SW, CS, OH, OW, N, KH, KW, stride=1, pad=0, src=None, src_pooled=None,
            src_argmax=None, bias=None, argmax=None, relu_mask=None, flip_taps=False, act=ACT_NONE, pool=False,
            dil=1, bn_src=None, bn_eps=1e-3, bn_momentum=0.99, bn_save=False):
    """Whole-image LDS convolution (small feature maps): forward (+bias/act/pool) or, with
    flip_taps and pad = K-1-pad, the data gradient of a stride-1 conv (w = Wt [cin][tap][cout]).
    The source may be un-pooled on load from (src_pooled, src_argmax), or dilated (``dil``: source
    pixel (y, x) at (y*dil, x*dil), zeros between - the data gradient of a stride-``dil`` conv).
    Returns y.  (The output BatchNorm statistics accumulated in the staged epilogue with a
    last-arriver fold measured 11-12 us slower per conv than the 4.5-6.7 us bn_stats pass it replaced -
    ResNet-20 1.312 vs 1.192 ms/step - and was removed in round 6: profiles/r6_resnet20_ostats_ab.txt.)"""
    if y.is_cuda:
        require().imgconv(src, src_pooled, src_argmax, w, bias, y, argmax, relu_mask, B, SH, SW, CS, OH, OW,
                          N, KH, KW, stride, pad, flip_taps, act, pool, dil, bn_src=bn_src, bn_eps=bn_eps,
                          bn_momentum=bn_momentum, bn_save=bn_save)
        return y
    if bn_src is not None:  # BN + ReLU formed on the source (the kernel does it while staging)
        src = _bn_src_ref(src, bn_src, bn_eps, bn_momentum, bn_save)
    s = src.float().view(B, SH, SW, CS) if src is not None else _unpooled_nhwc(src_pooled, src_argmax, B, SH, SW, CS)
    if dil > 1:
        sd = torch.zeros(B, SH * dil, SW * dil, CS)
        sd[:, ::dil, ::dil, :] = s
        s = sd
    wt = w.float().view(N, KH, KW, CS)
    if flip_taps:
        wt = wt.flip(1, 2)
    z = torch.nn.functional.conv2d(s.permute(0, 3, 1, 2), wt.permute(0, 3, 1, 2),
                                   bias.float() if bias is not None else None, stride=stride, padding=pad)
    z = z[:, :, :OH, :OW]
    z = _act_ref(z, act)
    if pool:
        p, idx = _pool_ref(z)
        y.view(-1)[:] = p.permute(0, 2, 3, 1).reshape(-1).to(y.dtype)
        if argmax is not None:
            argmax.view(-1)[:] = idx.permute(0, 2, 3, 1).reshape(-1).to(argmax.dtype)
        return y
    flat = z.permute(0, 2, 3, 1).reshape(-1)
    if relu_mask is not None:
        flat = flat * (relu_mask.reshape(-1).float() > 0)
    y.view(-1)[:] = flat.to(y.dtype)
    return y


def imgconv_shortcut(w, dx, g, sc_stride, *, src, **geom) -> bool:
    """Data gradient of a whole-image conv (flipped taps over ``src`` = dY, ``geom`` as for
    imgconv(flip_taps=True)) with the option-A shortcut's gradient added in the same launch:
    dx[:, ::s, ::s, :] += g[..., :N] (ops.shortcut_grad_add).  Returns True when the launch added it
    (the persistent kernel's LDS-staged epilogue); False: only dx was written and the caller adds
    the shortcut gradient.  The CPU path does both (the oracle)."""
    if dx.is_cuda:
        k = geom
        return bool(require().imgconv(src, None, None, w, None, dx, None, None, k["B"], k["SH"], k["SW"], k["CS"],
                                      k["OH"], k["OW"], k["N"], k["KH"], k["KW"], k.get("stride", 1), k.get("pad", 0),
                                      True, ACT_NONE, False, k.get("dil", 1), g, sc_stride))
    imgconv(w, dx, src=src, flip_taps=True, **geom)
    shortcut_grad_add(g, dx, sc_stride)
    return True


_WG_WS = {}


def wgrad_flush() -> int:
    """Launch every weight-gradient reduce queued by imgwgrad(defer=True) as ONE grouped launch on the
    current stream (each deferred call needs its own workspace).  CPU: nothing is ever deferred."""
    if available():
        return int(require().wgrad_flush())
    return 0


def wgrad_pending() -> int:
    """Deferred weight-gradient reduces queued on this thread and not yet flushed."""
    if available():
        return int(require().wgrad_pending())
    return 0


def wgrad_discard() -> int:
    """Drop this thread's queued deferred reduces (after an interrupted backward); returns how many."""
    if available():
        return int(require().wgrad_discard())
    return 0


def wgrad_ws_floats(N: int, KC: int) -> int:
    """Floats of the weight-gradient partial-sum workspace (256 workgroup slabs) - mirrors
    imgwgrad_ws_floats in csrc/kernels/imgwgrad_persist.hip (the register-layout slabs of the
    persistent kernel: 8 waves x CTW column tiles x MT row tiles x 64 lanes x 4, + db)."""
    MT, CTW = (4, 7) if N > 32 else (2, 9)
    return 256 * max(N * KC + N, 8 * CTW * MT * 256 + (N + 3) // 4 * 4)


def wgrad_workspace(device, numel):
    """Cached fp32 partial-sum buffer for the persistent weight-gradient kernel
    (per device, grown on demand; single-stream use)."""
    key = torch.device(device)
    ws = _WG_WS.get(key)
    if ws is None or ws.numel() < numel:
        if ws is not None:
            _WS_RETIRED.append((ws,))  # may be referenced by a captured graph
        ws = torch.empty(numel, device=key, dtype=torch.float32)
        _WG_WS[key] = ws
    return ws


def imgwgrad(src, dw, db, *, B, SH, SW, CS, OH, OW, N, KH, KW, stride=1, pad=0, dy=None, dy_pooled=None,
             dy_argmax=None, scale=1.0, workspace=None, max_blocks=0, bn_src=None, bn_eps=1e-3, defer=False):
    """dW[n][tap][c] += scale * sum_p dY[p][n] src[p*stride-pad+tap][c]; db += scale * sum dY.
    On the GPU the persistent kernel stores per-workgroup partials in `workspace`
    (default: a cached per-device buffer) and a second kernel sums them."""
    if dw.is_cuda:
        if workspace is None and (CS % 16 == 0 or CS == 1):
            workspace = wgrad_workspace(dw.device, wgrad_ws_floats(N, KH * KW * CS))
        require().imgwgrad(src, dy, dy_pooled, dy_argmax, dw, db, B, SH, SW, CS, OH, OW, N, KH, KW, stride, pad,
                           scale, workspace, max_blocks, bn_src=bn_src, bn_eps=bn_eps, defer=defer)
        return
    if bn_src is not None:  # the source's BN + ReLU (nothing saved: the forward did)
        src = _bn_src_ref(src, bn_src, bn_eps, 0.99, False)
    d = dy.float().view(B, OH, OW, N) if dy is not None else _unpooled_nhwc(dy_pooled, dy_argmax, B, OH, OW, N)
    gw = torch.nn.grad.conv2d_weight(src.float().view(B, SH, SW, CS).permute(0, 3, 1, 2), (N, CS, KH, KW),
                                     d.permute(0, 3, 1, 2), stride=stride, padding=pad)
    dw.view(-1)[:] += scale * gw.permute(0, 2, 3, 1).reshape(-1)
    if db is not None:
        db += scale * d.sum(dim=(0, 1, 2))


def conv_dgrad(dy, wt, dx, g, pooled=None, argmax=None, relu_mask=None, accumulate=False, bn_bwd=None,
               acc_src=None):
    """dX of an NHWC conv (wt = W laid out [C][KH][KW][Cout]); optional un-pool epilogue, or a
    ReLU mask (dx = mask > 0 ? dx : 0) when the consumer un-pools itself.  ``accumulate``:
    dx += dX (implicit-GEMM path: C and Cout multiples of 64); with ``acc_src = (src, bits)``
    dx = dX + src * bit instead (bits: relu_bits layout) - dx's old contents are not read.
    ``bn_bwd``: the consuming BatchNorm's backward statistics of the final dx, ``(x, y, mean,
    invstd, gamma, beta, stats, act)`` with ``bn_bwd_stats`` semantics - computed in the
    implicit-GEMM epilogue (no separate pass over dx and x), or by a statistics pass after the launch."""
    if dx.is_cuda:
        b = bn_bwd or (None,) * 7 + (0,)
        src, bits = acc_src or (None, None)
        require().conv_dgrad(dy, wt, dx, *_conv_geom_args(g), pooled, argmax, relu_mask, accumulate, *b, src, bits)
        return dx
    if acc_src is not None:
        src, bits = acc_src
        R, C = dx.numel() // dx.shape[-1], dx.shape[-1]
        dx.copy_((src.float().reshape(R, C) * _unbits(bits, R, C)).reshape(dx.shape).to(dx.dtype))
        return conv_dgrad(dy, wt, dx, g, pooled, argmax, relu_mask, True, bn_bwd)
    if bn_bwd is not None:
        conv_dgrad(dy, wt, dx, g, pooled, argmax, relu_mask, accumulate)
        x, y, mean, invstd, gamma, beta, stats, act = bn_bwd
        bn_bwd_stats(dx, y, x, mean, invstd, stats, act, gamma=gamma, beta=beta)
        return dx
    if accumulate:
        old = dx.float().clone()
        conv_dgrad(dy, wt, dx, g, pooled, argmax, relu_mask)
        dx.copy_((dx.float() + old).to(dx.dtype))
        return dx
    dyt = dy.float().view(g["B"], g["OH"], g["OW"], g["Cout"]).permute(0, 3, 1, 2)
    w = wt.float().view(g["C"], g["KH"], g["KW"], g["Cout"]).permute(3, 0, 1, 2)
    dxt = torch.nn.grad.conv2d_input((g["B"], g["C"], g["H"], g["W"]), w, dyt, stride=g["stride"], padding=g["pad"])
    flat = dxt.permute(0, 2, 3, 1).reshape(-1)
    if pooled is not None:
        _unpool_ref(flat, pooled, argmax, g["H"], g["W"], g["C"], dx)
    else:
        if relu_mask is not None:
            flat = flat * (relu_mask.reshape(-1).float() > 0)
        dx.view(-1)[:] = flat.to(dx.dtype)
    return dx


def conv_wgrad(dz, x, dw, db, g, scale=1.0):
    """dW[Cout][KH][KW][C] += scale * sum dz (x) im2col(x);  db += scale * sum dz."""
    if dw.is_cuda:
        require().conv_wgrad(dz, x, dw, db, *_conv_geom_args(g), scale)
        return dw
    xt = x.float().view(g["B"], g["H"], g["W"], g["C"]).permute(0, 3, 1, 2)
    dzt = dz.float().view(g["B"], g["OH"], g["OW"], g["Cout"]).permute(0, 3, 1, 2)
    gw = torch.nn.grad.conv2d_weight(xt, (g["Cout"], g["C"], g["KH"], g["KW"]), dzt, stride=g["stride"],
                                     padding=g["pad"])
    dw.view(-1)[:] += scale * gw.permute(0, 2, 3, 1).reshape(-1)
    if db is not None:
        db += scale * dzt.sum(dim=(0, 2, 3))
    return dw


def conv1_wgrad_pooled_f32(dp, argmax, x, dw, db, g, scale=1.0, dy=None):
    """MNIST conv1 weight gradient at fp32 (C = 1, 32 channels, 3x3 / 5x5 SAME, stride 1) from the
    POOLED gradient dp [B][H/2][W/2][32] (ReLU mask applied) and the pool's argmax bytes:
    dW += scale * sum_q dp[q][n] * x[argmax pixel of q + tap], db += scale * sum dp - the gradient of
    un-pool + conv_wgrad without the un-pooled tensor (GPU: conv1_wgrad_pooled_f32_kernel).  Other
    shapes, and the CPU oracle: un-pool into ``dy`` [B][H][W][32] (allocated if None) + conv_wgrad."""
    B, H, W, K = g["B"], g["H"], g["W"], g["KH"]
    if dw.is_cuda:
        ws = wgrad_workspace(dw.device, B * (32 * 25 + 32))
        if require().conv1_wgrad_pooled_f32(dp, argmax, x, dw, db, ws, B, H, W, K, scale):
            return dw
    if dy is None:
        dy = torch.empty(B, H, W, dp.shape[-1], device=dp.device, dtype=torch.float32)
    unpool_f32(dp, argmax, dy)
    return conv_wgrad(dy, x, dw, db, g, scale)


def unpool_f32(g, argmax, out):
    """out[B][2PH][2PW][C] (fp32) = g routed to the argmax position of each 2x2 window, zeros
    elsewhere (the max-pool gradient; the ReLU mask is already in g)."""
    B, PH, PW, C = g.shape
    if g.is_cuda:
        require().unpool_f32(g, argmax, out, B, PH, PW, C)
        return out
    _unpool_ref(g.reshape(-1).float(), torch.ones(B, PH, PW, C), argmax, PH, PW, C, out)
    return out


def transpose_taps_f32(w, out, O, T, C):
    """out[C][T][O] = w[O][T][C] (a conv weight laid out for its data gradient)."""
    if w.is_cuda:
        require().transpose_taps_f32(w, out, O, T, C)
        return out
    out.view(-1)[:] = w.reshape(O, T, C).permute(2, 1, 0).reshape(-1)
    return out


# -------------------------------------------------------------------- head
def head_xent_f32(h, w, b, labels, dz, dl, loss_sum, correct, logits=None, scale=1.0, inv_keep=1.0,
                  step_counter=None) -> bool:
    """fp32 fused classifier head (GPU, NC = 10, K = 1024): logits (optional), softmax-xent sums into
    loss_sum / correct, dlogit rows fp32 [B][NC] into ``dl``, dZ = (dlogit . W) * inv_keep * (h > 0),
    step_counter += 1 - one launch.  False (nothing done): CPU tensors or another shape - the caller
    runs the GEMM + softmax_xent + GEMM chain, which is also this kernel's oracle."""
    if not h.is_cuda:
        return False
    return bool(require().head_xent_f32(h, w, b, labels, dz, dl, loss_sum, correct, logits, scale, inv_keep,
                                        step_counter))


def head_xent(h, w, b, labels, dz, dl, loss_sum, correct, logits=None, scale=1.0, inv_keep=1.0, step_counter=None,
              parts=None):
    """Per-row classifier head: logits, softmax-xent (loss/correct sums), dlogit rows (bf16 [B][ld] into
    ``dl``) and dZ = (dlogit . W) * inv_keep * (h > 0).  dW/db come from a wgrad GEMM over ``dl``.
    ``step_counter`` (int64 [1], optional) is advanced by one.  ``parts`` (fp32 [>= 2 * ceil(B/4)],
    optional): the loss / hit sums of each 4-row workgroup are stored there instead of being added
    to ``loss_sum`` / ``correct``; ``head_wgrad(..., parts=...)`` folds them in (no atomics)."""
    if h.is_cuda:
        require().head_xent(h, w, b, labels, dz, dl, loss_sum, correct, logits, scale, inv_keep, step_counter, parts)
        return
    if step_counter is not None:
        step_counter += 1
    hf, wf = h.float(), w.float()
    lg = hf @ wf.t() + (b.float() if b is not None else 0)
    if logits is not None:
        logits.copy_(lg)
    lse = torch.logsumexp(lg, dim=1)
    lab = labels.long()
    rows = lse - lg.gather(1, lab[:, None])[:, 0]
    hits = (lg.argmax(1) == lab).float()
    if parts is not None:
        n = (len(lab) + 3) // 4
        pad = 4 * n - len(lab)
        parts[:n] = torch.nn.functional.pad(rows, (0, pad)).view(n, 4).sum(1)
        parts[n:2 * n] = torch.nn.functional.pad(hits, (0, pad)).view(n, 4).sum(1)
    else:
        if loss_sum is not None:
            loss_sum += rows.sum()
        if correct is not None:
            correct += hits.sum().to(correct.dtype)
    p = torch.softmax(lg, dim=1)
    p[torch.arange(len(lab)), lab] -= 1
    d = p * scale
    dl.zero_()
    dl[:, : d.shape[1]] = d.to(dl.dtype)
    g = (d @ wf) * (hf > 0).float() * inv_keep
    dz.copy_(g.to(dz.dtype))


def head_wgrad(dl, h, dw, db, nc, scale=1.0, parts=None, loss_sum=None, correct=None):
    """Classifier-head weight / bias gradient, stored: dw[c][:K] = scale * sum_b dl[b][c] h[b][:],
    db[c] = scale * sum_b dl[b][c] (one workgroup per 8 columns over the whole batch, fixed order).
    ``parts``: head_xent's per-workgroup loss / hit partials, summed by the bias workgroup into
    ``loss_sum`` / ``correct`` (needs ``db``)."""
    if h.is_cuda:
        require().head_wgrad(dl, h, dw, db, nc, scale, parts, loss_sum, correct)
        return
    d = dl[:, :nc].float()
    dw[:, : h.shape[1]] = (scale * (d.t() @ h.float())).to(dw.dtype)
    if db is not None:
        db.copy_((scale * d.sum(0)).to(db.dtype))
    if parts is not None:
        n = (h.shape[0] + 3) // 4
        loss_sum += parts[:n].sum()
        correct += parts[n:2 * n].sum().to(correct.dtype)


@contextlib.contextmanager
def gemm_group(anchor):
    """Grouped launch: the head_wgrad and glds-tile-12 one-split gemm calls inside the block are
    recorded and leave as ONE kernel launch at its end (head weight gradient, then the
    (KMAJ, RMAJ) and (RMAJ, RMAJ) GEMMs in recording order; any other mix launches one by one).
    fp32 small-tile GEMMs (the GAN / autoencoder layers): a (RMAJ, RMAJ) weight gradient and a
    (KMAJ, KMAJ) data gradient recorded in the block leave as one paired launch.
    CPU tensors: a no-op (the ops run eagerly)."""
    if not anchor.is_cuda:
        yield
        return
    lib = require()
    lib.gemm_group(anchor, True)
    try:
        yield
    finally:
        lib.gemm_group(anchor, False)


# --------------------------------------------------------------- optimizer
def opt_pack(segs, work, device_like):
    return require().opt_pack(segs, work, device_like)


def apply_gradients(kind, p, g, g16, gscale, s1, s2, lr, beta1, beta2, eps, momentum, rho, beta_pow, global_step,
                    gs_inc, done, blob, nseg, nwork, group=0):
    """group: 0 launch now, 1 queue, 2 queue + launch all queued optimizers as one grouped launch."""
    require().apply_gradients(kind, p, g, g16, gscale, s1, s2, lr, beta1, beta2, eps, momentum, rho, beta_pow,
                              global_step, gs_inc, done, blob, nseg, nwork, group)


# ------------------------------------------------------------- elementwise
def tallk_ws_floats(M: int, N: int, splits: int) -> int:
    """Partial-slab floats of wgrad_tallk (mirrors tallk_ws_floats in csrc/kernels/wgrad_tallk.hip)."""
    return splits * ((M + 1 + 15) // 16 * 16) * N


def wgrad_tallk(A, lda, B, ldb, M, N, K, out, ldc=None, bias=None, splits=32, scale=1.0, workspace=None):
    """Exact-fp32 weight gradient of a long reduction: out[m][n] = scale * sum_k A[k*lda+m] B[k*ldb+n]
    (stored), bias[n] = scale * sum_k B[k*ldb+n] (the LSTM kernel / bias gradient over T*B rows).
    GPU: K split over `splits` workgroups per 64-column slab + a fixed-order partial reduce."""
    ldc = N if ldc is None else ldc
    if out.is_cuda:
        ws = workspace if workspace is not None else wgrad_workspace(out.device, tallk_ws_floats(M, N, splits))
        require().wgrad_tallk(A, lda, B, ldb, M, N, K, out, ldc, bias, ws, splits, scale)
        return out
    a = torch.as_strided(A.reshape(-1), (K, M), (lda, 1)).double()
    b = torch.as_strided(B.reshape(-1), (K, N), (ldb, 1)).double()
    torch.as_strided(out.view(-1), (M, N), (ldc, 1)).copy_((scale * (a.t() @ b)).float())
    if bias is not None:
        bias.copy_((scale * b.sum(0)).float())
    return out


def seq_stage(x, xh, T, I, y_src, y_dst, zero=()):
    """LSTM batch staging (one launch on the GPU): xh[t, b, :I] = x[b, t*I:(t+1)*I] (image row t
    is timestep t), xh[0, :, I:] = 0 (h_{-1}), y_dst = y_src, and the tensors in ``zero`` (up to 4
    accumulators) cleared."""
    if xh.is_cuda:
        require().seq_stage(x.reshape(-1).contiguous(), xh, int(T), int(I), y_src.reshape(-1).contiguous(),
                            y_dst, list(zero))
        return
    B = xh.shape[1]
    xh[:, :, :I].copy_(x.reshape(B, T, I).transpose(0, 1))
    xh[0, :, I:].zero_()
    y_dst.copy_(y_src.reshape(y_dst.shape))
    for z in zero:
        z.zero_()


def gather_rows(src, dst, idx=None, labels_src=None, labels_dst=None, seed=0, counter=None, done=None, zero=(),
                onehot=None):
    """dst[b] = src[row(b)] (+ labels); ``zero``: up to 4 contiguous tensors cleared in the same
    launch (a step's accumulators), saving one fill kernel each; ``onehot``: f32 [B][ncls] one-hot
    rows of the gathered labels, also written in the same launch."""
    if dst.is_cuda:
        require().gather_rows(src, dst, idx, labels_src, labels_dst, seed, counter, done, list(zero), onehot)
        return dst
    for z in zero:
        z.zero_()
    if onehot is not None:
        onehot.zero_()
        onehot.scatter_(1, labels_src[idx.long()].long().unsqueeze(1), 1.0)
    assert idx is not None, "CPU gather needs explicit indices"
    rows = src[idx.long()]
    if src.dtype == torch.uint8:
        rows = rows.float() / 255.0
    dst.copy_(rows.reshape(dst.shape).to(dst.dtype))
    if labels_dst is not None:
        labels_dst.copy_(labels_src[idx.long()])
    return dst


def uniform_fill(out, lo, hi, seed=0, counter=None, done=None, copy=None):
    """out ~ U(lo, hi) from the device hash RNG (advances ``counter``); ``copy=(src, dst)``: an fp32
    copy issued in the same launch (batch staging next to the noise)."""
    if out.is_cuda:
        src, dst = copy if copy is not None else (None, None)
        require().uniform_fill(out, lo, hi, seed, counter, done, src, dst)
        return out
    if copy is not None:
        copy[1].copy_(copy[0])
    out.uniform_(lo, hi)
    return out


def cast_(src, dst):
    if dst.is_cuda:
        require().cast_(src, dst)
    else:
        dst.copy_(src.to(dst.dtype))
    return dst


def softmax_xent(logits, labels_i=None, labels_oh=None, scale=1.0, dlogits=None, loss_rows=None, loss_sum=None,
                 correct=None, probs=None):
    if logits.is_cuda:
        require().softmax_xent(logits, labels_i, labels_oh, scale, dlogits, loss_rows, loss_sum, correct, probs)
        return
    y = labels_oh.float() if labels_oh is not None else \
        torch.nn.functional.one_hot(labels_i.long(), logits.shape[1]).float()
    lse = torch.logsumexp(logits, 1, keepdim=True)
    p = torch.exp(logits - lse)
    rows = (y * (lse - logits)).sum(1)
    if dlogits is not None:
        dlogits.copy_((p - y) * scale)
    if loss_rows is not None:
        loss_rows.copy_(rows)
    if loss_sum is not None:
        loss_sum += rows.sum()
    if correct is not None:
        correct += (logits.argmax(1) == y.argmax(1)).sum().to(correct.dtype)
    if probs is not None:
        probs.copy_(p)


def gan_loss(d_real, d_fake, gen_loss, disc_loss, dz_real_disc, dz_fake_disc, dz_fake_gen, clamp_eps=0.0):
    if d_real.is_cuda:
        require().gan_loss(d_real, d_fake, gen_loss, disc_loss, dz_real_disc, dz_fake_disc, dz_fake_gen, clamp_eps)
        return
    B = d_real.numel()
    pr, pf = d_real.view(-1), d_fake.view(-1)
    if clamp_eps > 0:
        lr_, lf, lq = torch.log(pr.clamp_min(clamp_eps)), torch.log(pf.clamp_min(clamp_eps)), \
            torch.log((1 - pf).clamp_min(clamp_eps))
    else:
        lr_, lf, lq = torch.log(pr), torch.log(pf), torch.log(1 - pf)
    gen_loss.fill_(-lf.mean().item())
    disc_loss.fill_(-(lr_ + lq).mean().item())
    dz_real_disc.view(-1).copy_(-(1 - pr) / B)
    dz_fake_disc.view(-1).copy_(pf / B)
    dz_fake_gen.view(-1).copy_(-(1 - pf) / B)


def apply_wait_next(done, seen, segs: int):
    """The next apply_gradients launch's items of the var-list segments in bit mask ``segs`` wait (on the
    device) until ``done`` exceeds ``seen`` - a gradient produced on another stream that signals with
    epoch_signal(done) instead of a stream join; the launch's last workgroup advances ``seen``."""
    require().apply_wait_next(done, seen, int(segs))


def epoch_signal(ctr):
    """ctr += 1 on the current stream (after the producer a later apply_wait_next consumer waits for)."""
    require().epoch_signal(ctr)


def gan_head_ws_floats(B: int, DH: int) -> int:
    """Workspace floats of gan_disc_head (mirrors gan_head_ws_floats in csrc/kernels/head.hip)."""
    return max(1, min(256, (B + 3) // 4)) * 260 + 4


def gan_disc_head(d1, w, b, p, dlog, dlog_g, gw, gb, dd1, ddf, gen_loss, disc_loss, ws=None, clamp_eps=0.0) -> bool:
    """The GAN discriminator's output layer + both GAN losses + their gradients down to the hidden layer
    (csrc/kernels/head.h GanHeadArgs): d1 [2B][DH] (real rows, then fake rows), w = Wd2 [DH] (, b = bd2):
    p = sigmoid(d1 w + b) [2B], gen_loss / disc_loss (stored), dlog [2B], dlog_g [B], gw = dWd2 / gb = dbd2
    (stored), dd1 = dlog w^T relu'(d1) [2B][DH], ddf = dlog_g w^T relu'(d1_fake) [B][DH].  GPU: one launch
    (``ws``: gan_head_ws_floats zeroed floats, reused), returns False when the shape is not covered.  The CPU
    path is the fp32 oracle (the gemm + gan_loss chain it replaces)."""
    if d1.is_cuda:
        return bool(require().gan_disc_head(d1, w, b, p, dlog, dlog_g, gw, gb, dd1, ddf, gen_loss, disc_loss, ws,
                                            clamp_eps))
    B = d1.shape[0] // 2
    wv = w.reshape(-1)
    z = d1 @ wv + (b.reshape(()) if b is not None else 0.0)
    pp = torch.sigmoid(z)
    dl = torch.empty(2 * B, dtype=d1.dtype)
    dg = torch.empty(B, dtype=d1.dtype)
    gan_loss(pp[:B], pp[B:], gen_loss, disc_loss, dl[:B], dl[B:], dg, clamp_eps=clamp_eps)
    if p is not None:
        p.view(-1).copy_(pp)
    if dlog is not None:
        dlog.view(-1).copy_(dl)
    if dlog_g is not None:
        dlog_g.view(-1).copy_(dg)
    gw.view(-1).copy_(d1.t() @ dl)
    if gb is not None:
        gb.view(-1).copy_(dl.sum().reshape(1))
    mask = (d1 > 0).to(d1.dtype)
    dd1.copy_(dl[:, None] * wv[None, :] * mask)
    ddf.copy_(dg[:, None] * wv[None, :] * mask[B:])
    return True


MSE_WS_FLOATS = 132  # csrc/kernels/elementwise.h MSE_WS_FLOATS (128 partials + ticket)


def mse_sigmoid(y, t, loss, dz, ws=None):
    """loss = mean((y - t)^2), dz = d loss / d logit of y = sigmoid(logit).  ``ws`` (GPU, MSE_WS_FLOATS
    zeroed floats, reused every step): one launch whose last workgroup stores the loss (no memset node,
    bitwise-reproducible loss) instead of a memset + per-workgroup atomics."""
    if y.is_cuda:
        require().mse_sigmoid(y, t, loss, dz, ws)
        return
    n = y.numel()
    d = y - t
    loss.fill_((d * d).mean().item())
    dz.copy_(2 * d / n * y * (1 - y))


def dense_head(feat16, w, bias, y, logits, loss_sum, correct, dw, db, dfeat16, scale, w_fmajor=False,
               store=False, dl_out=None) -> bool:
    """A small dense classifier head, forward and backward in one launch (GPU: one workgroup; False when
    it does not fit): logits = feat W^T + b, softmax cross-entropy against one-hot y (loss_sum +=,
    correct +=), dlogits = (p - y) * scale, dw += dlogits^T feat, db += column sums, dfeat16 =
    dlogits W (in feat's dtype: bf16 or fp32).  ``w_fmajor``: W and dw are [F][NC] (a TF Variable of
    shape (in, out)) instead of [NC][F]; ``store``: dw / db are stored, not accumulated.  ``dl_out``
    (fp32 [B][NC]): the dlogits rows are written there, and dfeat16 may be None (the consumer forms it:
    lstm_seq_bwd(dl=...)).  The CPU path is the fp32 oracle."""
    if feat16.is_cuda:
        return bool(require().dense_head(feat16, w, bias, y, logits, loss_sum, correct, dw, db, dfeat16, scale,
                                         w_fmajor, store, dl_out))
    f = feat16.float()
    wf = w.float().t() if w_fmajor else w.float()   # [NC][F]
    lg = f @ wf.t() + (bias.float() if bias is not None else 0.0)
    if logits is not None:
        logits.copy_(lg)
    dl = torch.empty_like(lg)
    softmax_xent(lg, labels_oh=y, scale=scale, dlogits=dl, loss_sum=loss_sum, correct=correct)
    g = dl.t() @ f
    g = g.t() if w_fmajor else g
    if store:
        dw.copy_(g)
    else:
        dw += g
    if db is not None:
        if store:
            db.copy_(dl.sum(0))
        else:
            db += dl.sum(0)
    if dl_out is not None:
        dl_out.copy_(dl)
    if dfeat16 is not None:
        dfeat16.copy_((dl @ wf).to(dfeat16.dtype))
    return True


def colsum(x, M, N, ld, db, scale=1.0):
    if x.is_cuda:
        require().colsum(x, M, N, ld, db, scale)
        return
    idx = torch.arange(M).unsqueeze(1) * ld + torch.arange(N).unsqueeze(0)
    db += scale * x.reshape(-1).float()[idx].sum(0)


def act_grad(dy, y, dz, act):
    if dy.is_cuda:
        require().act_grad(dy, y, dz, act)
        return
    dz.copy_(dy * _act_grad_from_out_ref(y, act))


def bias_act(x, bias, out, act, keep=1.0, seed=0, counter=None):
    if x.is_cuda:
        require().bias_act(x, bias, out, act, keep, seed, counter)
        return
    v = x.float() + (bias.float() if bias is not None else 0)
    out.copy_(_act_ref(v, act).to(out.dtype))


# -------------------------------------------------------------------- LSTM
def lstm_cell_fwd(gates, act, c_prev, c, h_out, ld_h, forget_bias=1.0):
    """TF BasicLSTMCell step on pre-activation gates [B,4H] (order i, j, f, o)."""
    if gates.is_cuda:
        require().lstm_cell_fwd(gates, act, c_prev, c, h_out, ld_h, forget_bias)
        return
    H = c.shape[1]
    i, j, f, o = gates.split(H, dim=1)
    si, tj, sf, so = torch.sigmoid(i), torch.tanh(j), torch.sigmoid(f + forget_bias), torch.sigmoid(o)
    cn = (c_prev * sf if c_prev is not None else 0) + si * tj
    c.copy_(cn)
    act.copy_(torch.cat([si, tj, sf, so], dim=1))
    h_out.copy_(torch.tanh(cn) * so)  # h_out is a [B, H] (possibly strided) view


def lstm_cell_bwd(act, c_prev, c, dh, dh2, dc_next, dgates, dc_prev):
    if act.is_cuda:
        require().lstm_cell_bwd(act, c_prev, c, dh, dh2, dc_next, dgates, dc_prev)
        return
    H = c.shape[1]
    si, tj, sf, so = act.split(H, dim=1)
    d = (dh if dh is not None else 0) + (dh2 if dh2 is not None else 0)
    tc = torch.tanh(c)
    dc = (dc_next if dc_next is not None else 0) + d * so * (1 - tc * tc)
    cp = c_prev if c_prev is not None else torch.zeros_like(c)
    dgates.copy_(torch.cat([dc * tj * si * (1 - si), dc * si * (1 - tj * tj), dc * cp * sf * (1 - sf),
                            d * tc * so * (1 - so)], dim=1))
    dc_prev.copy_(dc * sf)


# ------------------------------------------------------------- batch norm
# NHWC bf16 activations viewed as [R][C]; stats are fp32 [2][C] accumulators the
# caller zeroes: forward (sum, sum of squares) of x - x[row 0] (per-channel shift),
# backward (sum g, sum g*xhat).
def _rows(t):
    return t.reshape(-1, t.shape[-1]).float()


def bn_stats(x, stats):
    if x.is_cuda:
        require().bn_stats(x, stats)
        return
    r = _rows(x)
    C = r.shape[1]
    d = r - r[0]  # shifted by row 0 (as the kernel) against E[x^2]-E[x]^2 cancellation
    stats[:C] += d.sum(0)
    stats[C:] += (d * d).sum(0)


def _bn_params(stats, R, eps, shift):
    C = stats.numel() // 2
    d = stats[:C] / R
    var = (stats[C:] / R - d * d).clamp_min(0)
    return shift + d, torch.rsqrt(var + eps), var


def _shortcut_view(res, OH, OW, C, rstride):
    """option-A shortcut read: res[:, ::s, ::s, :] zero-padded to C channels (NHWC fp32)."""
    r = res.float()[:, ::rstride, ::rstride, :][:, :OH, :OW, :]
    if r.shape[-1] < C:
        r = torch.nn.functional.pad(r, (0, C - r.shape[-1]))
    return r


def bn_apply(x, stats, gamma, beta, out, *, mean=None, invstd=None, moving_mean=None, moving_var=None, eps=1e-3,
             momentum=0.99, act=ACT_RELU, res=None, rstride=1, mask_out=None, res_bn=None):
    """out = act(gamma * (x - mean) * invstd + beta [+ shortcut(res)]) with batch statistics from
    ``stats``; stores mean/invstd and updates the moving averages (TF momentum convention).
    ``mask_out`` (ReLU): uint8 [R][C/8] bit mask of out > 0, which the backward ops take in place
    of ``y`` (``relu_bits``).  ``res_bn`` = [stats, gamma, beta, mean, invstd, moving_mean,
    moving_var] of the residual's own BatchNorm (a projection shortcut, no activation): ``res`` is
    then that BN's raw input, normalised here exactly as its own bn_apply would store it, and that
    BN's mean / invstd / moving averages are saved / updated here too."""
    OH, OW = (x.shape[1], x.shape[2]) if x.dim() == 4 else (1, 1)
    if x.is_cuda:
        require().bn_apply(x, stats, gamma, beta, mean, invstd, moving_mean, moving_var, eps, momentum, act, res,
                           rstride, OH, OW, out, mask_out, res_bn)
        return out
    if res_bn is not None:
        rs, rg, rb, rm, ri, rmm, rmv = res_bn
        r_out = torch.empty_like(res)
        bn_apply(res, rs, rg, rb, r_out, mean=rm, invstd=ri, moving_mean=rmm, moving_var=rmv, eps=eps,
                 momentum=momentum, act=ACT_NONE)
        res = r_out
    r = _rows(x)
    R, C = r.shape
    m, inv, var = _bn_params(stats, R, eps, r[0])
    if mean is not None:
        mean.copy_(m)
    if invstd is not None:
        invstd.copy_(inv)
    if moving_mean is not None:
        unb = var * R / max(R - 1, 1)
        moving_mean.mul_(momentum).add_(m * (1 - momentum))
        moving_var.mul_(momentum).add_(unb * (1 - momentum))
    y = (r - m) * inv * gamma.float() + beta.float()
    if res is not None:
        y = y + _shortcut_view(res, OH, OW, C, rstride).reshape(R, C)
    out.copy_(_act_ref(y, act).reshape(out.shape).to(out.dtype))
    if mask_out is not None:
        mask_out.copy_(relu_bits(out))
    return out


def relu_bits(y):
    """uint8 [R][C/8] bit mask of y > 0 (bit e of byte (r, j) = channel 8 j + e) - the layout
    bn_apply(mask_out=...) writes."""
    r = _rows(y) > 0
    R, C = r.shape
    w = (1 << torch.arange(8, device=r.device, dtype=torch.int32))
    return (r.reshape(R, C // 8, 8).to(torch.int32) * w).sum(-1).to(torch.uint8).reshape(-1)


def _unbits(m, R, C):
    e = torch.arange(8, device=m.device, dtype=torch.int32)
    return ((m.reshape(R, C // 8, 1).to(torch.int32) >> e) & 1).reshape(R, C).bool()


def bn_infer(x, gamma, beta, moving_mean, moving_var, out, *, eps=1e-3, act=ACT_RELU, res=None, rstride=1):
    """Inference-mode BatchNorm (TF ``training=False``): out = act(gamma * (x - moving_mean) *
    rsqrt(moving_var + eps) + beta [+ shortcut(res)]); nothing is updated."""
    OH, OW = (x.shape[1], x.shape[2]) if x.dim() == 4 else (1, 1)
    if x.is_cuda:
        require().bn_infer(x, gamma, beta, moving_mean, moving_var, eps, act, res, rstride, OH, OW, out)
        return out
    r = _rows(x)
    R, C = r.shape
    inv = torch.rsqrt(moving_var.float() + eps)
    y = (r - moving_mean.float()) * inv * gamma.float() + beta.float()
    if res is not None:
        y = y + _shortcut_view(res, OH, OW, C, rstride).reshape(R, C)
    out.copy_(_act_ref(y, act).reshape(out.shape).to(out.dtype))
    return out


def _masked_grad(dy, y, act, x=None, mean=None, invstd=None, gamma=None, beta=None):
    g = _rows(dy)
    if act != ACT_NONE:
        if y is None:  # ReLU mask recomputed from the pre-normalisation input (no residual in the forward)
            scale = gamma.float() * invstd
            pre = _rows(x) * scale + (beta.float() - mean * scale)
            return g * (pre > 0)
        if y.dtype == torch.uint8:  # bn_apply's bit mask of the ReLU output
            return g * _unbits(y, g.shape[0], g.shape[1])
        g = g * _act_grad_from_out_ref(_rows(y), act)
    return g


def bn_bwd_stats(dy, y, x, mean, invstd, stats, act=ACT_RELU, gamma=None, beta=None, res_bn=None):
    """stats += (sum g, sum g*xhat), g = dy*act'(y).  With y=None and act=ReLU the mask is
    recomputed from x (the forward had no residual add): pass gamma and beta.  ``res_bn`` = [x2,
    mean2, invstd2, stats2] (y a uint8 ReLU bit mask): the same pass also adds (sum g, sum g*xhat2)
    into stats2 - a projection shortcut's BN, whose gradient is this g."""
    if x.is_cuda:
        require().bn_bwd_stats(dy, y, x, mean, invstd, stats, act, gamma, beta, res_bn)
        return
    g = _masked_grad(dy, y, act, x, mean, invstd, gamma, beta)
    xh = (_rows(x) - mean) * invstd
    C = g.shape[1]
    stats[:C] += g.sum(0)
    stats[C:] += (g * xh).sum(0)
    if res_bn is not None:
        x2, m2, i2, s2 = res_bn
        s2[:C] += g.sum(0)
        s2[C:] += (g * ((_rows(x2) - m2) * i2)).sum(0)


def bn_bwd_apply(dy, y, x, mean, invstd, gamma, stats, dx, *, act=ACT_RELU, dres=None, dgamma=None, dbeta=None,
                 beta=None):
    """dx = gamma*invstd*(g - mean(g) - xhat*mean(g*xhat)), g = dy*act'(y); dgamma/dbeta += sums;
    dres = g (gradient of an added shortcut).  y=None + beta: ReLU mask from x (see bn_bwd_stats)."""
    if x.is_cuda:
        require().bn_bwd_apply(dy, y, x, mean, invstd, gamma, stats, act, dx, dres, dgamma, dbeta, beta)
        return dx
    g = _masked_grad(dy, y, act, x, mean, invstd, gamma, beta)
    R, C = g.shape
    xh = (_rows(x) - mean) * invstd
    d = gamma.float() * invstd * (g - stats[:C] / R - xh * stats[C:] / R)
    dx.copy_(d.reshape(dx.shape).to(dx.dtype))
    if dres is not None:
        dres.copy_(g.reshape(dres.shape).to(dres.dtype))
    if dgamma is not None:
        dgamma += stats[C:]
    if dbeta is not None:
        dbeta += stats[:C]
    return dx


def shortcut_grad_add(g, dx, stride=1):
    """dx[:, ::s, ::s, :XC] += g[..., :XC] (gradient of the option-A identity shortcut)."""
    if dx.is_cuda:
        require().shortcut_grad_add(g, dx, stride)
        return dx
    XC = dx.shape[-1]
    OH, OW = g.shape[1], g.shape[2]
    v = dx[:, ::stride, ::stride, :][:, :OH, :OW, :]
    v.copy_((v.float() + g[..., :XC].float()).to(dx.dtype))
    return dx


def gap_fwd(x, y):
    if x.is_cuda:
        require().gap_fwd(x, y)
        return y
    y.copy_(x.float().mean(dim=(1, 2)).reshape(y.shape).to(y.dtype))
    return y


def gap_bwd(dy, dx):
    if dx.is_cuda:
        require().gap_bwd(dy, dx)
        return dx
    B, H, W, C = dx.shape
    dx.copy_((dy.float().reshape(B, 1, 1, C) / (H * W)).expand(B, H, W, C).to(dx.dtype))
    return dx


def maxpool3_fwd(x, y, am):
    """3x3 / stride 2 / pad 1 max pool (NHWC) with the window argmax (0..8, first max wins)."""
    if x.is_cuda:
        require().maxpool3_fwd(x, y, am)
        return y
    B, H, W, C = x.shape
    xp = torch.nn.functional.pad(x.float().permute(0, 3, 1, 2), (1, 1, 1, 1), value=-3.0e38)
    cols = torch.nn.functional.unfold(xp, 3, stride=2)  # [B, C*9, L]
    OH, OW = y.shape[1], y.shape[2]
    cols = cols.view(B, C, 9, OH * OW)
    v, i = cols.max(dim=2)
    y.copy_(v.view(B, C, OH, OW).permute(0, 2, 3, 1).to(y.dtype))
    am.copy_(i.view(B, C, OH, OW).permute(0, 2, 3, 1).to(am.dtype))
    return y


def bn_relu_pool3(x, stats, gamma, beta, y, am, *, mean=None, invstd=None, moving_mean=None, moving_var=None,
                  eps=1e-3, momentum=0.99):
    """bn_apply(act=ReLU) + maxpool3_fwd in one pass: the pooled output ``y`` and argmax ``am`` of
    the normalised map, which is never stored; mean / invstd / moving averages as bn_apply.  Bit-
    identical to the two-op sequence (the ResNet-50 stem)."""
    if x.is_cuda:
        require().bn_relu_pool3(x, stats, gamma, beta, mean, invstd, moving_mean, moving_var, eps, momentum, y, am)
        return y
    h = torch.empty_like(x)
    bn_apply(x, stats, gamma, beta, h, mean=mean, invstd=invstd, moving_mean=moving_mean, moving_var=moving_var,
             eps=eps, momentum=momentum, act=ACT_RELU)
    return maxpool3_fwd(h, y, am)


def pool3_bn_bwd(dp, am, x, mean, invstd, gamma, beta, stats, dx, *, dgamma=None, dbeta=None):
    """maxpool3_bwd + bn_bwd_stats + bn_bwd_apply (ReLU mask recomputed from x) without the unpooled
    gradient: ``dp`` / ``am`` are the pooled gradient and argmax, ``x`` the BN input, ``stats`` the
    zeroed [2][C] backward accumulators; dx, dgamma / dbeta (+=) as bn_bwd_apply (the ResNet-50 stem)."""
    if dx.is_cuda:
        require().pool3_bn_bwd(dp, am, x, mean, invstd, gamma, beta, stats, dx, dgamma, dbeta)
        return dx
    d = maxpool3_bwd(dp, am, torch.empty_like(x))
    bn_bwd_stats(d, None, x, mean, invstd, stats, ACT_RELU, gamma=gamma, beta=beta)
    bn_bwd_apply(d, None, x, mean, invstd, gamma, stats, dx, act=ACT_RELU, dgamma=dgamma, dbeta=dbeta, beta=beta)
    return dx


def maxpool3_bwd(dy, am, dx):
    if dx.is_cuda:
        require().maxpool3_bwd(dy, am, dx)
        return dx
    B, H, W, C = dx.shape
    OH, OW = dy.shape[1], dy.shape[2]
    cols = torch.zeros(B, C, 9, OH * OW)
    g = dy.float().permute(0, 3, 1, 2).reshape(B, C, 1, OH * OW)
    cols.scatter_(2, am.long().permute(0, 3, 1, 2).reshape(B, C, 1, OH * OW), g)
    d = torch.nn.functional.fold(cols.view(B, C * 9, OH * OW), (H + 2, W + 2), 3, stride=2)[:, :, 1:H + 1, 1:W + 1]
    dx.copy_(d.permute(0, 2, 3, 1).to(dx.dtype))
    return dx
