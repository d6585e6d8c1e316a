#pragma once
// Per-channel BatchNorm (training) coefficients shared by every kernel that forms a BN output:
// bn_apply / bn_finalize / bn_relu_pool3 (norm.hip) and the whole-image convs that apply a BN + ReLU
// to their source while staging it (imgconv_persist.hip / imgwgrad_persist.hip, BnSrc).  One
// definition, no multiply-add contraction: every kernel gets the same bits for mean / invstd /
// scale / shift whatever inlining context the compiler sees.
#include "common.h"

namespace dtfe {

// statistics [2][C] = (sum (x-K), sum (x-K)^2) with the shift K = x[row 0][c] (bn_stats)
__device__ __forceinline__ void bn_chan_params(const bf16* x, const float* stats, long R, int C, float eps, int c,
                                               float& mean, float& invstd) {
#pragma clang fp contract(off)
  const float inv_r = 1.f / (float)R;
  const float d = stats[c] * inv_r;
  mean = bf2f(x[c]) + d;
  const float var = fmaxf(stats[C + c] * inv_r - d * d, 0.f);
  invstd = rsqrtf(var + eps);
}

// Partial statistics (K_t, s_t = sum (y - K_t), q_t = sum (y - K_t)^2) over n_t rows moved to the
// shift K and added to (S, Q):  s = s_t + n_t d,  q = q_t + 2 d s_t + n_t d^2  with d = K_t - K
__device__ __forceinline__ void bn_shift_fold(float Kt, float st, float qt, float nt, float K, float& S, float& Q) {
  const float d = Kt - K;
  S += st + nt * d;
  Q += qt + 2.f * d * st + nt * d * d;
}

// saved statistics + moving averages of one channel (TF: unbiased batch variance)
__device__ __forceinline__ void bn_save_chan(long R, float eps, float momentum, int c, float mean, float invstd,
                                             float* smean, float* sinv, float* mm, float* mv) {
#pragma clang fp contract(off)
  if (smean) smean[c] = mean;
  if (sinv) sinv[c] = invstd;
  if (mm) {
    const float var = 1.f / (invstd * invstd) - eps;
    const float unb = R > 1 ? var * (float)R / (float)(R - 1) : var;
    mm[c] = mm[c] * momentum + mean * (1.f - momentum);
    mv[c] = mv[c] * momentum + unb * (1.f - momentum);
  }
}

// A BatchNorm + ReLU formed on a conv's source while the conv stages it (ResNet-20: bn1 on conv2's
// forward and weight-gradient loads - its bn_apply pass is never launched).  The source tensor is
// the BN's raw input x; stats == nullptr: no transform.
struct BnSrc {
  const float* stats;                       // [2][C] shifted sums (K = x[row 0])
  const float* gamma; const float* beta;
  float* mean; float* invstd;               // saved batch statistics (workgroup 0; nullptr: not saved)
  float* moving_mean; float* moving_var;    // updated by workgroup 0 when non-null
  long R; float eps, momentum;
};

// (scale, shift) of channels [c0, c0 + 8) - bn_apply's expressions
__device__ __forceinline__ void bn_src_coeffs(const BnSrc& b, const bf16* x, int C, int c0, float (&sc)[8],
                                              float (&sh)[8]) {
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    float mean, invstd;
    bn_chan_params(x, b.stats, b.R, C, b.eps, c0 + e, mean, invstd);
    sc[e] = b.gamma[c0 + e] * invstd;
    sh[e] = bn_shift(b.beta[c0 + e], mean, sc[e]);
  }
}

// workgroup 0 of the conv that owns the BN's forward: saved statistics + moving averages
__device__ __forceinline__ void bn_src_save(const BnSrc& b, const bf16* x, int C, int nthreads) {
  if (!b.mean) return;
  for (int c = threadIdx.x; c < C; c += nthreads) {
    float mean, invstd;
    bn_chan_params(x, b.stats, b.R, C, b.eps, c, mean, invstd);
    bn_save_chan(b.R, b.eps, b.momentum, c, mean, invstd, b.mean, b.invstd, b.moving_mean, b.moving_var);
  }
}

// relu(bn(x)) of one 16-B chunk (8 channels), rounded to bf16 as bn_apply stores it
__device__ __forceinline__ u32x4_t bn_relu_chunk(const u32x4_t v, const float (&sc)[8], const float (&sh)[8]) {
  u32x4_t o;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float lo = apply_act(bn_affine(__uint_as_float(v[i] << 16), sc[2 * i], sh[2 * i]), ACT_RELU);
    const float hi = apply_act(bn_affine(__uint_as_float(v[i] & 0xffff0000u), sc[2 * i + 1], sh[2 * i + 1]), ACT_RELU);
    o[i] = pack_bf16x2(lo, hi);
  }
  return o;
}

}  // namespace dtfe
