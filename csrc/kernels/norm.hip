// BatchNorm (training), option-A residual shortcuts, global average pool and
// 3x3/s2 max pool for the ResNet models - see norm.h.
//
// Layout: NHWC bf16 viewed as [R][C] rows with C % 8 == 0 and C/8 a power of
// two; every thread owns one 16-byte chunk (8 channels) of a row, so loads and
// stores are 16 B vectors and a warp-wide load covers whole 128 B lines.
// Channel statistics are reduced per workgroup through LDS and then added to
// the [2][C] accumulators with one atomic per channel and workgroup.
#include "norm.h"
#include "bn_chan.h"

#include <cstdlib>
#include <stdexcept>

namespace dtfe {

namespace {

constexpr int NT = 256;

__device__ __forceinline__ void unpack8(const u32x4_t v, float (&f)[8]) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = bf2f((bf16)(v[i] & 0xffffu));
    f[2 * i + 1] = bf2f((bf16)(v[i] >> 16));
  }
}

__device__ __forceinline__ u32x4_t pack8(const float (&f)[8]) {
  u32x4_t v;
#pragma unroll
  for (int i = 0; i < 4; ++i) v[i] = pack_bf16x2(f[2 * i], f[2 * i + 1]);
  return v;
}

__device__ __forceinline__ float act_fwd(float x, int act) { return apply_act(x, act); }

// per-thread (row slot, chunk) decomposition of a block of NT threads
struct Slots {
  int tpr, rpp, chunk, slot;
  __device__ Slots(int C) {
    tpr = C / 8;
    rpp = NT / tpr;
    chunk = threadIdx.x % tpr;
    slot = threadIdx.x / tpr;
  }
};

// block-reduce s[8], q[8] of every thread onto channels and add them to stats[0..C), stats[C..2C)
__device__ void reduce_stats(const float (&s)[8], const float (&q)[8], int C, float* stats) {
  extern __shared__ float red[];  // [rpp][2][C]
  const Slots S(C);
  float* mine = red + S.slot * 2 * C;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    mine[S.chunk * 8 + e] = s[e];
    mine[C + S.chunk * 8 + e] = q[e];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < 2 * C; c += NT) {
    float v = 0.f;
    for (int r = 0; r < S.rpp; ++r) v += red[r * 2 * C + c];
    atomicAdd(stats + c, v);
  }
}

// Every row loop below keeps U independent 16-B loads in flight per thread (all
// issued before any of them is consumed): the kernels are HBM-latency bound
// otherwise (one outstanding load per thread ~ 1 KB per wave).
constexpr int U_STATS = 8, U_APPLY = 4;

__device__ __forceinline__ u32x4_t ld16(const bf16* p) { return *reinterpret_cast<const u32x4_t*>(p); }

// Statistics are accumulated around a per-channel shift K = x[row 0][c] (sum (x-K), sum (x-K)^2):
// the one-pass E[x^2] - E[x]^2 form loses the variance to cancellation when |mean| >> std.
// Rows past the end re-read row 0 (= K), which contributes exactly zero.
__global__ __launch_bounds__(NT) void bn_stats_kernel(BnArgs a) {
  const Slots S(a.C);
  float k[8];
  unpack8(ld16(a.x + S.chunk * 8), k);
  float s[8] = {}, q[8] = {};
  const long step = (long)gridDim.x * S.rpp * U_STATS;
  for (long r0 = (long)blockIdx.x * S.rpp * U_STATS + S.slot; r0 < a.R; r0 += step) {
    u32x4_t v[U_STATS];
#pragma unroll
    for (int u = 0; u < U_STATS; ++u) {
      const long r = r0 + (long)u * S.rpp;
      v[u] = ld16(a.x + (r < a.R ? r : 0) * a.C + S.chunk * 8);
    }
#pragma unroll
    for (int u = 0; u < U_STATS; ++u) {
      float f[8];
      unpack8(v[u], f);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float d = f[e] - k[e];
        s[e] += d;
        q[e] += d * d;
      }
    }
  }
  reduce_stats(s, q, a.C, a.stats);
}

// (no fp contraction here: every kernel that recomputes a channel's mean / invstd - bn_apply's
// workgroup 0 and its threads, bn_finalize, bn_relu_pool3 - must get the same bits whatever inlining
// context the compiler sees; contracted `x[c] + stats[c] * inv_r` in one of them made the folded and
// the materialised BN outputs differ in the last place)
__device__ __forceinline__ void chan_params_of(const bf16* x, const float* stats, long R, int C, float eps, int c,
                                               float& mean, float& invstd) {
  bn_chan_params(x, stats, R, C, eps, c, mean, invstd);  // (bn_chan.h: shared with the whole-image convs)
}

__device__ __forceinline__ void chan_params(const BnArgs& a, int c, float& mean, float& invstd) {
  chan_params_of(a.x, a.stats, a.R, a.C, a.eps, c, mean, invstd);
}

// saved statistics + moving averages of one channel (TF: unbiased batch variance)
__device__ __forceinline__ void save_chan(const BnArgs& a, int c, float mean, float invstd, float* smean,
                                          float* sinv, float* mm, float* mv) {
  bn_save_chan(a.R, a.eps, a.momentum, c, mean, invstd, smean, sinv, mm, mv);
}

__device__ __forceinline__ long res_offset(const BnArgs& a, long r, int chunk, bool identity) {
  if (identity) return r * a.C + chunk * 8;
  const long hw = (long)a.OH * a.OW, b = r / hw;
  const int p = (int)(r - b * hw), oy = p / a.OW, ox = p - oy * a.OW;
  return ((b * a.RH + (long)oy * a.rstride) * a.RW + (long)ox * a.rstride) * a.RC + chunk * 8;
}

// INFER: TF inference mode - (x - moving_mean) * rsqrt(moving_variance + eps), nothing updated.
// (A runtime flag in the training kernel's channel setup made hipcc unswitch and re-shape the row
// loop: bn_apply 53 -> 123 us per ResNet-50 call.  The two modes are separate instantiations.)
// ACTC: the activation as a compile-time constant (ACT_NONE / ACT_RELU), or -1 for the runtime a.act;
// RES: a residual source is given.  (The runtime forms of both put a branch on every value of the
// row loop: 2.4k static VALU instructions against ~0.8k for the ReLU / residual instance.)
// RBN: the residual goes through its own BatchNorm first (BnArgs.r_stats: a projection shortcut)
template <bool INFER, int ACTC, bool RES, bool RBN = false>
__global__ __launch_bounds__(NT) void bn_apply_kernel(BnArgs a) {
  const Slots S(a.C);
  if (!INFER && blockIdx.x == 0) {  // saved statistics + moving averages (TF: unbiased batch variance)
    for (int c = threadIdx.x; c < a.C; c += NT) {
      float mean, invstd;
      chan_params(a, c, mean, invstd);
      save_chan(a, c, mean, invstd, a.mean, a.invstd, a.moving_mean, a.moving_var);
      if (RBN) {
        chan_params_of(a.res, a.r_stats, a.R, a.C, a.eps, c, mean, invstd);
        save_chan(a, c, mean, invstd, a.r_mean, a.r_invstd, a.r_moving_mean, a.r_moving_var);
      }
    }
  }
  float rscale[8], rshift[8];
  if constexpr (RBN) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int c = S.chunk * 8 + e;
      float mean, invstd;
      chan_params_of(a.res, a.r_stats, a.R, a.C, a.eps, c, mean, invstd);
      rscale[e] = a.r_gamma[c] * invstd;
      rshift[e] = bn_shift(a.r_beta[c], mean, rscale[e]);
    }
  }
  float scale[8], shift[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int c = S.chunk * 8 + e;
    float mean, invstd;
    if constexpr (INFER) {
      mean = a.moving_mean[c];
      invstd = rsqrtf(a.moving_var[c] + a.eps);
    } else {
      chan_params(a, c, mean, invstd);
    }
    scale[e] = a.gamma[c] * invstd;
    shift[e] = bn_shift(a.beta[c], mean, scale[e]);
  }
  const bool res_identity = RES && a.rstride == 1 && a.RC == a.C && a.RH == a.OH && a.RW == a.OW;
  const bool res_chunk = RES && S.chunk * 8 < a.RC;
  const long step = (long)gridDim.x * S.rpp * U_APPLY;
  for (long r0 = (long)blockIdx.x * S.rpp * U_APPLY + S.slot; r0 < a.R; r0 += step) {
    u32x4_t v[U_APPLY], w[U_APPLY];
#pragma unroll
    for (int u = 0; u < U_APPLY; ++u) {
      const long r = r0 + (long)u * S.rpp;
      const long rr = r < a.R ? r : 0;
      v[u] = ld16(a.x + rr * a.C + S.chunk * 8);
      if (res_chunk) w[u] = ld16(a.res + res_offset(a, rr, S.chunk, res_identity));
    }
#pragma unroll
    for (int u = 0; u < U_APPLY; ++u) {
      const long r = r0 + (long)u * S.rpp;
      float f[8];
      unpack8(v[u], f);
#pragma unroll
      for (int e = 0; e < 8; ++e) f[e] = bn_affine(f[e], scale[e], shift[e]);
      if (res_chunk) {
        float g[8];
        unpack8(w[u], g);
        if constexpr (RBN) {  // the shortcut BN's output as its own bn_apply (ACT_NONE) would store it
#pragma unroll
          for (int e = 0; e < 8; ++e) g[e] = act_fwd(bn_affine(g[e], rscale[e], rshift[e]), ACT_NONE);
          unpack8(pack8(g), g);
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) f[e] += g[e];
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) f[e] = act_fwd(f[e], ACTC >= 0 ? ACTC : a.act);
      if (r < a.R) {
        const u32x4_t o = pack8(f);
        *reinterpret_cast<u32x4_t*>(a.out + r * a.C + S.chunk * 8) = o;
        if (a.mask_out) {  // of the stored bf16 values: the backward's y > 0, bit for bit
          uint32_t bits = 0;
#pragma unroll
          for (int e = 0; e < 4; ++e)
            bits |= ((o[e] & 0x7fffu) != 0 && !(o[e] & 0x8000u) ? 1u : 0u) << (2 * e) |
                    ((o[e] & 0x7fff0000u) != 0 && !(o[e] & 0x80000000u) ? 1u : 0u) << (2 * e + 1);
          a.mask_out[r * (a.C / 8) + S.chunk] = (uint8_t)bits;
        }
      }
    }
  }
}

// Backward activation mask, as a compile-time mode MM (the runtime form branched on every value):
//   MM_NONE  no activation: g = dy
//   MM_X     ReLU recomputed from x as (gamma*invstd*x + (beta - mean*gamma*invstd)) > 0 - bit-identical
//            to the forward's pre-activation (same fma on the same saved statistics), one tensor read
//            cheaper (y == nullptr)
//   MM_YRELU ReLU mask from the stored output y (a residual was added before the ReLU)
//   MM_YACT  act'(y) of the stored output for the runtime a.act (sigmoid / tanh)
//   MM_BITS  ReLU mask from the forward's 1-bit mask (ymask)
enum { MM_NONE = 0, MM_X = 1, MM_YRELU = 2, MM_YACT = 3, MM_BITS = 4 };

__host__ __device__ inline int mask_mode(const BnArgs& a) {
  if (a.act == ACT_NONE) return MM_NONE;
  if (a.ymask && a.act == ACT_RELU) return MM_BITS;
  if (a.y == nullptr && a.act == ACT_RELU) return MM_X;
  return a.act == ACT_RELU ? MM_YRELU : MM_YACT;
}

struct BwdMask {
  float scale[8], shift[8];
  __device__ BwdMask(const BnArgs& a, int chunk, bool from_x) {
    if (from_x) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int c = chunk * 8 + e;
        scale[e] = a.gamma[c] * a.invstd[c];
        shift[e] = bn_shift(a.beta[c], a.mean[c], scale[e]);
      }
    }
  }
};

// g = dy * act'(.) for 8 channels, from loaded dy / y / x chunks
template <int MM>
__device__ __forceinline__ void masked_grad(const BnArgs& a, const BwdMask& M, const u32x4_t dyv, const u32x4_t yv,
                                            const float (&x)[8], float (&g)[8]) {
  unpack8(dyv, g);
  if constexpr (MM == MM_BITS) {  // (yv[0] carries the mask byte)
#pragma unroll
    for (int e = 0; e < 8; ++e) g[e] = (yv[0] >> e) & 1u ? g[e] : 0.f;
  } else if constexpr (MM == MM_X) {
#pragma unroll
    for (int e = 0; e < 8; ++e) g[e] = bn_affine(x[e], M.scale[e], M.shift[e]) > 0.f ? g[e] : 0.f;
  } else if constexpr (MM == MM_YRELU) {
    float y[8];
    unpack8(yv, y);
#pragma unroll
    for (int e = 0; e < 8; ++e) g[e] *= y[e] > 0.f ? 1.f : 0.f;  // = act_grad_from_out(y, ReLU), bit for bit
  } else if constexpr (MM == MM_YACT) {
    float y[8];
    unpack8(yv, y);
#pragma unroll
    for (int e = 0; e < 8; ++e) g[e] *= act_grad_from_out(y[e], a.act);
  }
}

// DUAL (MM_BITS only): also the backward statistics of a projection shortcut's BN (BnArgs.res /
// r_mean / r_invstd -> r_stats) from the same g - that BN's own statistics pass re-read dy and the mask
template <int MM, bool DUAL = false>
__global__ __launch_bounds__(NT) void bn_bwd_stats_kernel(BnArgs a) {
  const Slots S(a.C);
  const BwdMask M(a, S.chunk, MM == MM_X);
  constexpr bool need_y = MM == MM_YRELU || MM == MM_YACT;
  float mean[8], invstd[8], rmean[8], rinv[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    mean[e] = a.mean[S.chunk * 8 + e];
    invstd[e] = a.invstd[S.chunk * 8 + e];
    if (DUAL) {
      rmean[e] = a.r_mean[S.chunk * 8 + e];
      rinv[e] = a.r_invstd[S.chunk * 8 + e];
    }
  }
  constexpr int U = DUAL ? U_STATS / 2 : U_STATS;  // (registers: the shortcut input's loads ride along)
  float s[8] = {}, q[8] = {}, q2[8] = {};
  const long step = (long)gridDim.x * S.rpp * U;
  for (long r0 = (long)blockIdx.x * S.rpp * U + S.slot; r0 < a.R; r0 += step) {
    u32x4_t dv[U], xv[U], yv[U], zv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long r = r0 + (long)u * S.rpp;
      const long off = (r < a.R ? r : 0) * a.C + S.chunk * 8;
      dv[u] = ld16(a.dy + off);
      xv[u] = ld16(a.x + off);
      if (need_y) yv[u] = ld16(a.y + off);
      if (MM == MM_BITS) yv[u][0] = a.ymask[off >> 3];
      if (DUAL) zv[u] = ld16(a.res + off);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const float live = (r0 + (long)u * S.rpp) < a.R ? 1.f : 0.f;
      float g[8], x[8];
      unpack8(xv[u], x);
      masked_grad<MM>(a, M, dv[u], yv[u], x, g);
      float z[8];
      if (DUAL) unpack8(zv[u], z);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float gl = g[e] * live;
        s[e] += gl;
        q[e] += gl * (x[e] - mean[e]) * invstd[e];
        if (DUAL) q2[e] += gl * (z[e] - rmean[e]) * rinv[e];
      }
    }
  }
  reduce_stats(s, q, a.C, a.stats);
  if constexpr (DUAL) {
    __syncthreads();  // the LDS scratch is reused
    reduce_stats(s, q2, a.C, a.r_stats);
  }
}

template <int MM>
__global__ __launch_bounds__(NT) void bn_bwd_apply_kernel(BnArgs a) {
  const Slots S(a.C);
  if (blockIdx.x == 0) {
    for (int c = threadIdx.x; c < a.C; c += NT) {
      if (a.dbeta) a.dbeta[c] += a.stats[c];
      if (a.dgamma) a.dgamma[c] += a.stats[a.C + c];
    }
  }
  const BwdMask M(a, S.chunk, MM == MM_X);
  constexpr bool need_y = MM == MM_YRELU || MM == MM_YACT;
  const float inv_r = 1.f / (float)a.R;
  float mean[8], invstd[8], k[8], sg[8], sgx[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int c = S.chunk * 8 + e;
    mean[e] = a.mean[c];
    invstd[e] = a.invstd[c];
    k[e] = a.gamma[c] * invstd[e];
    sg[e] = a.stats[c] * inv_r;
    sgx[e] = a.stats[a.C + c] * inv_r;
  }
  const long step = (long)gridDim.x * S.rpp * U_APPLY;
  for (long r0 = (long)blockIdx.x * S.rpp * U_APPLY + S.slot; r0 < a.R; r0 += step) {
    u32x4_t dv[U_APPLY], xv[U_APPLY], yv[U_APPLY];
#pragma unroll
    for (int u = 0; u < U_APPLY; ++u) {
      const long r = r0 + (long)u * S.rpp;
      const long off = (r < a.R ? r : 0) * a.C + S.chunk * 8;
      dv[u] = ld16(a.dy + off);
      xv[u] = ld16(a.x + off);
      if (need_y) yv[u] = ld16(a.y + off);
      if (MM == MM_BITS) yv[u][0] = a.ymask[off >> 3];
    }
#pragma unroll
    for (int u = 0; u < U_APPLY; ++u) {
      const long r = r0 + (long)u * S.rpp;
      if (r >= a.R) continue;
      const long off = r * a.C + S.chunk * 8;
      float g[8], x[8], dx[8];
      unpack8(xv[u], x);
      masked_grad<MM>(a, M, dv[u], yv[u], x, g);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float xh = (x[e] - mean[e]) * invstd[e];
        dx[e] = k[e] * (g[e] - sg[e] - xh * sgx[e]);
      }
      *reinterpret_cast<u32x4_t*>(a.out + off) = pack8(dx);
      if (a.dres) *reinterpret_cast<u32x4_t*>(a.dres + off) = pack8(g);
    }
  }
}

// Statistics kernels: few enough workgroups that the per-channel atomics stay cheap
// (about 2 per CU), each looping over U_STATS-row batches.  Apply kernels: one U_APPLY-row
// batch per thread, as many workgroups as that takes (no atomics to amortise).
// Workgroup cap: every workgroup adds 2C atomics, and with 512 of them those serialized adds were a
// visible part of the small layers' time.  ResNet-50 B=256 sweep (profiles/r4_bn_stats_grid.txt):
// 256 beats 512 on every shape, 128 is better still below ~64 MB of activations and worse above.
// ResNet-20 shapes (2-8 MB) re-swept in round 5: 128 / 256 / 512 / 1024 all within 0.1 us except
// stage 1 (128: 6.4 us, more: 7.5) - the same-address atomics, not the grid, set the floor
// (profiles/r5_resnet20_kernels.txt).
int stats_grid(long R, int C) {
  const long rows_per_block = (long)(NT / (C / 8)) * U_STATS;
  long g = (R + rows_per_block - 1) / rows_per_block;
  const long cap = R * C * 2 <= (64L << 20) ? 128 : 256;
  if (g > cap) g = cap;
  return g < 1 ? 1 : (int)g;
}

int apply_grid(long R, int C) {
  const long rows_per_block = (long)(NT / (C / 8)) * U_APPLY;
  long g = (R + rows_per_block - 1) / rows_per_block;
  if (g > (1L << 20)) g = 1L << 20;
  return g < 1 ? 1 : (int)g;
}

void check(const BnArgs& a) {
  const int t = a.C / 8;
  if (a.C % 8 || t > NT || (t & (t - 1))) throw std::runtime_error("bn: C must be 8 * 2^k <= 2048");
}

__global__ void shortcut_grad_kernel(const bf16* g, bf16* dx, int B, int OH, int OW, int C, int XH, int XW, int XC,
                                     int stride) {
  const int cpr = XC / 8;
  const long n = (long)B * OH * OW * cpr;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const long row = i / cpr;
    const int ch = (int)(i - row * cpr) * 8;
    const long hw = (long)OH * OW, b = row / hw;
    const int p = (int)(row - b * hw), oy = p / OW, ox = p - oy * OW;
    const long xo = ((b * XH + (long)oy * stride) * XW + (long)ox * stride) * XC + ch;
    float a8[8], b8[8];
    unpack8(*reinterpret_cast<const u32x4_t*>(g + row * C + ch), a8);
    unpack8(*reinterpret_cast<const u32x4_t*>(dx + xo), b8);
#pragma unroll
    for (int e = 0; e < 8; ++e) b8[e] += a8[e];
    *reinterpret_cast<u32x4_t*>(dx + xo) = pack8(b8);
  }
}

// one workgroup per image: threads = (chunk, pixel lane); pixel lanes reduce through LDS
__global__ __launch_bounds__(256) void gap_fwd_kernel(const bf16* x, bf16* y, int B, int HW, int C) {
  __shared__ float red[256 * 8];
  const int cpr = C / 8;  // power of two <= 256
  const int lanes = 256 / cpr, chunk = threadIdx.x % cpr, pl = threadIdx.x / cpr;
  const long b = blockIdx.x;
  float s[8] = {};
  for (int p = pl; p < HW; p += lanes) {
    float f[8];
    unpack8(*reinterpret_cast<const u32x4_t*>(x + (b * HW + p) * C + chunk * 8), f);
#pragma unroll
    for (int e = 0; e < 8; ++e) s[e] += f[e];
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) red[threadIdx.x * 8 + e] = s[e];
  __syncthreads();
  if (pl == 0) {
    for (int l = 1; l < lanes; ++l)
#pragma unroll
      for (int e = 0; e < 8; ++e) s[e] += red[(l * cpr + chunk) * 8 + e];
#pragma unroll
    for (int e = 0; e < 8; ++e) s[e] *= 1.f / (float)HW;
    *reinterpret_cast<u32x4_t*>(y + b * C + chunk * 8) = pack8(s);
  }
}

__global__ void gap_bwd_kernel(const bf16* dy, bf16* dx, int B, int HW, int C) {
  const int cpr = C / 8;
  const long n = (long)B * HW * cpr;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const long row = i / cpr;
    const int ch = (int)(i - row * cpr) * 8;
    const long b = row / HW;
    float f[8];
    unpack8(*reinterpret_cast<const u32x4_t*>(dy + b * C + ch), f);
#pragma unroll
    for (int e = 0; e < 8; ++e) f[e] *= 1.f / (float)HW;
    *reinterpret_cast<u32x4_t*>(dx + row * C + ch) = pack8(f);
  }
}

// 3x3/s2/p1 max pool, one thread per (output pixel, 8-channel chunk): 16-B loads of every tap,
// argmax (tap 0..8, first max wins) packed 8 bytes per chunk.
__global__ __launch_bounds__(256) void maxpool3_fwd_kernel(const bf16* x, bf16* y, uint8_t* am, int B, int H, int W,
                                                           int C, int OH, int OW) {
  const int cpr = C / 8;
  const long n = (long)B * OH * OW * cpr;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const long row = i / cpr;
    const int ch = (int)(i - row * cpr) * 8;
    const long hw = (long)OH * OW, b = row / hw;
    const int p = (int)(row - b * hw), oy = p / OW, ox = p - oy * OW;
    u32x4_t v[9];
    bool ok[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int iy = oy * 2 - 1 + t / 3, ix = ox * 2 - 1 + t % 3;
      ok[t] = iy >= 0 && iy < H && ix >= 0 && ix < W;
      if (ok[t]) v[t] = ld16(x + ((b * H + iy) * W + ix) * C + ch);
    }
    float best[8];
    uint32_t arg[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) { best[e] = -3.0e38f; arg[e] = 0; }
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      if (!ok[t]) continue;
      float f[8];
      unpack8(v[t], f);
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (f[e] > best[e]) { best[e] = f[e]; arg[e] = t; }
    }
    *reinterpret_cast<u32x4_t*>(y + row * C + ch) = pack8(best);
    u32x2_t packed = {arg[0] | arg[1] << 8 | arg[2] << 16 | arg[3] << 24, arg[4] | arg[5] << 8 | arg[6] << 16 | arg[7] << 24};
    *reinterpret_cast<u32x2_t*>(am + row * C + ch) = packed;
  }
}

// BatchNorm apply + ReLU + 3x3 / stride-2 / pad-1 max pool in ONE pass (the ResNet-50 stem): each
// thread normalises the 9 window pixels of its pooled pixel x 8 channels straight from the conv
// output and keeps the max and its argmax.  The bn_apply -> maxpool3_fwd pair wrote the 112x112
// normalised map (411 MB bf16 at B=256) and read it back; the backward never needs it (the stem BN
// recomputes its ReLU mask from x, maxpool3_bwd reads the argmax).  Every value is formed exactly as
// bn_apply forms it (same scale / shift, bf16 rounding) and compared as maxpool3_fwd compares it
// (first max wins), so y / am are bit-identical to the pair's.  Workgroup 0 also stores mean /
// invstd and updates the moving averages, as bn_apply does.
__global__ __launch_bounds__(256) void bn_relu_pool3_kernel(BnArgs a, bf16* y, uint8_t* am, int B, int H, int W,
                                                            int OH, int OW) {
  const int C = a.C, cpr = C / 8;
  if (blockIdx.x == 0) {
    for (int c = threadIdx.x; c < C; c += 256) {
      float mean, invstd;
      chan_params(a, c, mean, invstd);
      if (a.mean) a.mean[c] = mean;
      if (a.invstd) a.invstd[c] = invstd;
      if (a.moving_mean) {
        const float var = 1.f / (invstd * invstd) - a.eps;
        const float unb = a.R > 1 ? var * (float)a.R / (float)(a.R - 1) : var;
        a.moving_mean[c] = a.moving_mean[c] * a.momentum + mean * (1.f - a.momentum);
        a.moving_var[c] = a.moving_var[c] * a.momentum + unb * (1.f - a.momentum);
      }
    }
  }
  // the grid stride is a multiple of cpr (the launcher checks 256 % cpr == 0): one chunk per thread
  const int ch = (int)(((long)blockIdx.x * 256 + threadIdx.x) % cpr) * 8;
  float scale[8], shift[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    float mean, invstd;
    chan_params(a, ch + e, mean, invstd);
    scale[e] = a.gamma[ch + e] * invstd;
    shift[e] = bn_shift(a.beta[ch + e], mean, scale[e]);
  }
  const long n = (long)B * OH * OW * cpr;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const long row = i / cpr;
    const long hw = (long)OH * OW, b = row / hw;
    const int p = (int)(row - b * hw), oy = p / OW, ox = p - oy * OW;
    u32x4_t v[9];
    bool ok[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int iy = oy * 2 - 1 + t / 3, ix = ox * 2 - 1 + t % 3;
      ok[t] = iy >= 0 && iy < H && ix >= 0 && ix < W;
      if (ok[t]) v[t] = ld16(a.x + ((b * H + iy) * W + ix) * C + ch);
    }
    float best[8];
    uint32_t arg[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) { best[e] = -3.0e38f; arg[e] = 0; }
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      if (!ok[t]) continue;
      float f[8];
      unpack8(v[t], f);
#pragma unroll
      for (int e = 0; e < 8; ++e) f[e] = act_fwd(bn_affine(f[e], scale[e], shift[e]), ACT_RELU);
      unpack8(pack8(f), f);  // the bf16 value bn_apply would have stored
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (f[e] > best[e]) { best[e] = f[e]; arg[e] = t; }
    }
    *reinterpret_cast<u32x4_t*>(y + row * C + ch) = pack8(best);
    u32x2_t packed = {arg[0] | arg[1] << 8 | arg[2] << 16 | arg[3] << 24, arg[4] | arg[5] << 8 | arg[6] << 16 | arg[7] << 24};
    *reinterpret_cast<u32x2_t*>(am + row * C + ch) = packed;
  }
}

// one thread per (2x2 input cell, 8-channel chunk): input rows 2k, 2k+1 are covered only by window
// rows k (both) and k+1 (the odd row), columns likewise, so the thread issues the <= 4 window loads
// (dy 16 B + argmax 8 B each) up front and writes 4 input pixels; each pixel sums its windows in
// (oy, ox) order, as a per-pixel gather would
__global__ __launch_bounds__(256) void maxpool3_bwd_kernel(const bf16* dy, const uint8_t* am, bf16* dx, int B, int H,
                                                           int W, int C, int OH, int OW) {
  const int cpr = C / 8;
  const int QH = (H + 1) / 2, QW = (W + 1) / 2;
  const long n = (long)B * QH * QW * cpr;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const long cell = i / cpr;
    const int ch = (int)(i - cell * cpr) * 8;
    const long qhw = (long)QH * QW, b = cell / qhw;
    const int p = (int)(cell - b * qhw), k = p / QW, j = p - k * QW;
    u32x4_t d[2][2];
    u32x2_t m[2][2];
    bool ok[2][2];
#pragma unroll
    for (int a2 = 0; a2 < 2; ++a2)
#pragma unroll
      for (int c2 = 0; c2 < 2; ++c2) {
        const int oy = k + a2, ox = j + c2;
        ok[a2][c2] = oy < OH && ox < OW;
        if (ok[a2][c2]) {
          const long o = ((b * OH + oy) * OW + ox) * C + ch;
          d[a2][c2] = ld16(dy + o);
          m[a2][c2] = *reinterpret_cast<const u32x2_t*>(am + o);
        }
      }
#pragma unroll
    for (int yi = 0; yi < 2; ++yi) {
      const int iy = 2 * k + yi;
      if (iy >= H) continue;
#pragma unroll
      for (int xi = 0; xi < 2; ++xi) {
        const int ix = 2 * j + xi;
        if (ix >= W) continue;
        float g[8] = {};
#pragma unroll
        for (int a2 = 0; a2 < 2; ++a2) {
          const int ty = yi - 2 * a2 + 1;  // tap row of (iy) in window row k + a2
          if (ty < 0) continue;
#pragma unroll
          for (int c2 = 0; c2 < 2; ++c2) {
            const int tx = xi - 2 * c2 + 1;
            if (tx < 0 || !ok[a2][c2]) continue;
            const uint32_t t = (uint32_t)(ty * 3 + tx);
            float dv[8];
            unpack8(d[a2][c2], dv);
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const uint32_t ae = ((e < 4 ? m[a2][c2][0] : m[a2][c2][1]) >> (8 * (e & 3))) & 0xffu;
              if (ae == t) g[e] += dv[e];
            }
          }
        }
        *reinterpret_cast<u32x4_t*>(dx + ((b * H + iy) * W + ix) * C + ch) = pack8(g);
      }
    }
  }
}

// maxpool3_bwd fused into the stem BatchNorm's backward (ReLU mask recomputed from x, MM_X): one
// thread per (2x2 input cell, 8-channel chunk) as in maxpool3_bwd - the <= 4 pooled windows (dy 16 B
// + argmax 8 B each) and the 4 pixels of x are loaded up front, each pixel's upstream gradient is
// summed in maxpool3_bwd's (oy, ox) order and rounded to bf16 exactly as that kernel stores it, then
// masked and either reduced into the statistics (STATS) or turned into dx (apply).  The 112x112
// unpooled gradient (411 MB bf16 at B=256) is never stored or read back.  The apply half is bit-
// identical to maxpool3_bwd + bn_bwd_apply on the same statistics.
template <bool STATS>
__global__ __launch_bounds__(NT) void pool3_bn_bwd_kernel(BnArgs a, const uint8_t* am, int B, int H, int W, int OH,
                                                          int OW) {
  const int C = a.C, cpr = C / 8;
  if (!STATS && blockIdx.x == 0) {
    for (int c = threadIdx.x; c < C; c += NT) {
      if (a.dbeta) a.dbeta[c] += a.stats[c];
      if (a.dgamma) a.dgamma[c] += a.stats[C + c];
    }
  }
  const int chunk = threadIdx.x % cpr;  // the grid stride is a multiple of cpr (NT % cpr == 0)
  const int ch = chunk * 8;
  const BwdMask M(a, chunk, true);
  const float inv_r = 1.f / (float)a.R;
  float mean[8], invstd[8], k[8], sg[8], sgx[8], s[8] = {}, q[8] = {};
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    mean[e] = a.mean[ch + e];
    invstd[e] = a.invstd[ch + e];
    if (!STATS) {
      k[e] = a.gamma[ch + e] * invstd[e];
      sg[e] = a.stats[ch + e] * inv_r;
      sgx[e] = a.stats[C + ch + e] * inv_r;
    }
  }
  const int QH = (H + 1) / 2, QW = (W + 1) / 2;
  const long n = (long)B * QH * QW * cpr;
  for (long i = (long)blockIdx.x * NT + threadIdx.x; i < n; i += (long)gridDim.x * NT) {
    const long cell = i / cpr;
    const long qhw = (long)QH * QW, b = cell / qhw;
    const int p = (int)(cell - b * qhw), kq = p / QW, jq = p - kq * QW;
    u32x4_t d[2][2], xv[2][2];
    u32x2_t m[2][2];
    bool ok[2][2];
#pragma unroll
    for (int a2 = 0; a2 < 2; ++a2)
#pragma unroll
      for (int c2 = 0; c2 < 2; ++c2) {
        const int oy = kq + a2, ox = jq + c2;
        ok[a2][c2] = oy < OH && ox < OW;
        if (ok[a2][c2]) {
          const long o = ((b * OH + oy) * OW + ox) * C + ch;
          d[a2][c2] = ld16(a.dy + o);
          m[a2][c2] = *reinterpret_cast<const u32x2_t*>(am + o);
        }
        const int iy = 2 * kq + a2, ix = 2 * jq + c2;
        if (iy < H && ix < W) xv[a2][c2] = ld16(a.x + ((b * H + iy) * W + ix) * C + ch);
      }
#pragma unroll
    for (int yi = 0; yi < 2; ++yi) {
      const int iy = 2 * kq + yi;
      if (iy >= H) continue;
#pragma unroll
      for (int xi = 0; xi < 2; ++xi) {
        const int ix = 2 * jq + xi;
        if (ix >= W) continue;
        float g[8] = {};
#pragma unroll
        for (int a2 = 0; a2 < 2; ++a2) {
          const int ty = yi - 2 * a2 + 1;  // tap row of (iy) in window row kq + a2
          if (ty < 0) continue;
#pragma unroll
          for (int c2 = 0; c2 < 2; ++c2) {
            const int tx = xi - 2 * c2 + 1;
            if (tx < 0 || !ok[a2][c2]) continue;
            const uint32_t t = (uint32_t)(ty * 3 + tx);
            float dv[8];
            unpack8(d[a2][c2], dv);
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const uint32_t ae = ((e < 4 ? m[a2][c2][0] : m[a2][c2][1]) >> (8 * (e & 3))) & 0xffu;
              if (ae == t) g[e] += dv[e];
            }
          }
        }
        float x[8];
        unpack8(xv[yi][xi], x);
        masked_grad<MM_X>(a, M, pack8(g), u32x4_t{0u, 0u, 0u, 0u}, x, g);  // bf16 dy as maxpool3_bwd stores it
        if constexpr (STATS) {
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            s[e] += g[e];
            q[e] += g[e] * (x[e] - mean[e]) * invstd[e];
          }
        } else {
          float dx[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float xh = (x[e] - mean[e]) * invstd[e];
            dx[e] = k[e] * (g[e] - sg[e] - xh * sgx[e]);
          }
          *reinterpret_cast<u32x4_t*>(a.out + ((b * H + iy) * W + ix) * C + ch) = pack8(dx);
        }
      }
    }
  }
  if constexpr (STATS) reduce_stats(s, q, C, a.stats);
}

int ew_grid(long n) {
  long g = (n + 255) / 256;
  if (g > 65536) g = 65536;
  return g < 1 ? 1 : (int)g;
}

}  // namespace

void launch_bn_stats(const BnArgs& a, hipStream_t s) {
  check(a);
  const size_t lds = (size_t)(NT / (a.C / 8)) * 2 * a.C * sizeof(float);
  hipLaunchKernelGGL(bn_stats_kernel, dim3(stats_grid(a.R, a.C)), dim3(NT), lds, s, a);
}

void launch_bn_apply(const BnArgs& a, hipStream_t s) {
  check(a);
  if (a.infer && (!a.moving_mean || !a.moving_var)) throw std::runtime_error("bn_apply: inference needs the moving averages");
  if (a.res && (a.RC % 8 || a.RC > a.C)) throw std::runtime_error("bn_apply: residual channels");
  const dim3 g(apply_grid(a.R, a.C)), b(NT);
  const bool res = a.res != nullptr;
  if (a.r_stats) {  // projection shortcut BN folded into this residual apply (training, ReLU, same shape)
    if (!res || a.infer || a.act != ACT_RELU || a.rstride != 1 || a.RC != a.C || a.RH != a.OH || a.RW != a.OW ||
        !a.r_gamma || !a.r_beta)
      throw std::runtime_error("bn_apply: a residual BN needs training mode, ReLU and a same-shape raw residual");
    hipLaunchKernelGGL((bn_apply_kernel<false, ACT_RELU, true, true>), g, b, 0, s, a);
    return;
  }
  const int act = a.act == ACT_NONE || a.act == ACT_RELU ? a.act : -1;
#define BN_APPLY(INF, ACT)                                                              \
  do {                                                                                  \
    if (res) hipLaunchKernelGGL((bn_apply_kernel<INF, ACT, true>), g, b, 0, s, a);      \
    else hipLaunchKernelGGL((bn_apply_kernel<INF, ACT, false>), g, b, 0, s, a);         \
  } while (0)
  if (a.infer) {
    if (act == ACT_RELU) BN_APPLY(true, ACT_RELU);
    else if (act == ACT_NONE) BN_APPLY(true, ACT_NONE);
    else BN_APPLY(true, -1);
  } else {
    if (act == ACT_RELU) BN_APPLY(false, ACT_RELU);
    else if (act == ACT_NONE) BN_APPLY(false, ACT_NONE);
    else BN_APPLY(false, -1);
  }
#undef BN_APPLY
}

void check_bwd(const BnArgs& a) {
  check(a);
  if (a.act != ACT_NONE && !a.y && !(a.ymask && a.act == ACT_RELU) && (a.act != ACT_RELU || !a.gamma || !a.beta))
    throw std::runtime_error("bn_bwd: the activation mask needs y, or (ReLU) gamma and beta");
}

void launch_bn_bwd_stats(const BnArgs& a, hipStream_t s) {
  check_bwd(a);
  if (a.r_stats && (mask_mode(a) != MM_BITS || !a.res || !a.r_mean || !a.r_invstd))
    throw std::runtime_error("bn_bwd_stats: the shortcut BN's statistics ride along only with a bit mask (res, r_mean, r_invstd)");
  const size_t lds = (size_t)(NT / (a.C / 8)) * 2 * a.C * sizeof(float);
  const dim3 g(stats_grid(a.R, a.C)), b(NT);
  switch (mask_mode(a)) {
    case MM_NONE: hipLaunchKernelGGL(bn_bwd_stats_kernel<MM_NONE>, g, b, lds, s, a); break;
    case MM_X: hipLaunchKernelGGL(bn_bwd_stats_kernel<MM_X>, g, b, lds, s, a); break;
    case MM_YRELU: hipLaunchKernelGGL(bn_bwd_stats_kernel<MM_YRELU>, g, b, lds, s, a); break;
    case MM_BITS:
      if (a.r_stats) hipLaunchKernelGGL((bn_bwd_stats_kernel<MM_BITS, true>), g, b, lds, s, a);
      else hipLaunchKernelGGL(bn_bwd_stats_kernel<MM_BITS>, g, b, lds, s, a);
      break;
    default: hipLaunchKernelGGL(bn_bwd_stats_kernel<MM_YACT>, g, b, lds, s, a); break;
  }
}

void launch_bn_bwd_apply(const BnArgs& a, hipStream_t s) {
  check_bwd(a);
  const dim3 g(apply_grid(a.R, a.C)), b(NT);
  switch (mask_mode(a)) {
    case MM_NONE: hipLaunchKernelGGL(bn_bwd_apply_kernel<MM_NONE>, g, b, 0, s, a); break;
    case MM_X: hipLaunchKernelGGL(bn_bwd_apply_kernel<MM_X>, g, b, 0, s, a); break;
    case MM_YRELU: hipLaunchKernelGGL(bn_bwd_apply_kernel<MM_YRELU>, g, b, 0, s, a); break;
    case MM_BITS: hipLaunchKernelGGL(bn_bwd_apply_kernel<MM_BITS>, g, b, 0, s, a); break;
    default: hipLaunchKernelGGL(bn_bwd_apply_kernel<MM_YACT>, g, b, 0, s, a); break;
  }
}

void launch_shortcut_grad_add(const bf16* g, bf16* dx, int B, int OH, int OW, int C, int XH, int XW, int XC,
                              int stride, hipStream_t s) {
  if (XC % 8 || C % 8 || XC > C) throw std::runtime_error("shortcut_grad_add: channels");
  hipLaunchKernelGGL(shortcut_grad_kernel, dim3(ew_grid((long)B * OH * OW * XC / 8)), dim3(256), 0, s, g, dx, B, OH,
                     OW, C, XH, XW, XC, stride);
}

void launch_gap_fwd(const bf16* x, bf16* y, int B, int HW, int C, hipStream_t s) {
  const int t = C / 8;
  if (C % 8 || t > 256 || (t & (t - 1))) throw std::runtime_error("gap: C must be 8 * 2^k <= 2048");
  hipLaunchKernelGGL(gap_fwd_kernel, dim3(B), dim3(256), 0, s, x, y, B, HW, C);
}

void launch_gap_bwd(const bf16* dy, bf16* dx, int B, int HW, int C, hipStream_t s) {
  if (C % 8) throw std::runtime_error("gap: C % 8");
  hipLaunchKernelGGL(gap_bwd_kernel, dim3(ew_grid((long)B * HW * C / 8)), dim3(256), 0, s, dy, dx, B, HW, C);
}

void launch_maxpool3_fwd(const bf16* x, bf16* y, uint8_t* am, int B, int H, int W, int C, int OH, int OW,
                         hipStream_t s) {
  if (C % 8) throw std::runtime_error("maxpool3: C % 8");
  hipLaunchKernelGGL(maxpool3_fwd_kernel, dim3(ew_grid((long)B * OH * OW * C / 8)), dim3(256), 0, s, x, y, am, B, H,
                     W, C, OH, OW);
}

void launch_pool3_bn_bwd(const BnArgs& a, const uint8_t* am, int B, int H, int W, int OH, int OW, hipStream_t s) {
  check(a);
  if (NT % (a.C / 8) || a.R != (long)B * H * W || a.act != ACT_RELU || !a.gamma || !a.beta || a.y || a.ymask ||
      a.dres || OH != (H + 1) / 2 || OW != (W + 1) / 2)
    throw std::runtime_error("pool3_bn_bwd: ReLU mask from x (gamma, beta), NT % (C/8) == 0, 3x3/s2/p1 pool geometry");
  const long n = (long)B * ((H + 1) / 2) * ((W + 1) / 2) * (a.C / 8);
  const size_t lds = (size_t)(NT / (a.C / 8)) * 2 * a.C * sizeof(float);
  // statistics: a few workgroups per CU (2C atomics each; cf. stats_grid), apply: the whole range
  long gs = (n + NT - 1) / NT;
  if (gs > 1024) gs = 1024;
  hipLaunchKernelGGL(pool3_bn_bwd_kernel<true>, dim3((unsigned)gs), dim3(NT), lds, s, a, am, B, H, W, OH, OW);
  hipLaunchKernelGGL(pool3_bn_bwd_kernel<false>, dim3(ew_grid(n)), dim3(NT), 0, s, a, am, B, H, W, OH, OW);
}

void launch_bn_relu_pool3(const BnArgs& a, bf16* y, uint8_t* am, int B, int H, int W, int OH, int OW,
                          hipStream_t s) {
  if (a.C % 8 || 256 % (a.C / 8) || a.R != (long)B * H * W || a.infer)
    throw std::runtime_error("bn_relu_pool3: training mode, C % 8 == 0, 256 % (C / 8) == 0, R == B*H*W");
  hipLaunchKernelGGL(bn_relu_pool3_kernel, dim3(ew_grid((long)B * OH * OW * a.C / 8)), dim3(256), 0, s, a, y, am, B, H,
                     W, OH, OW);
}

void launch_maxpool3_bwd(const bf16* dy, const uint8_t* am, bf16* dx, int B, int H, int W, int C, int OH, int OW,
                         hipStream_t s) {
  if (C % 8) throw std::runtime_error("maxpool3: C % 8");
  hipLaunchKernelGGL(maxpool3_bwd_kernel, dim3(ew_grid((long)B * ((H + 1) / 2) * ((W + 1) / 2) * C / 8)), dim3(256), 0,
                     s, dy, am, dx, B, H, W, C, OH, OW);
}

}  // namespace dtfe
