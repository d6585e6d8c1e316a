// NHWC bf16 convolution as implicit GEMM on MFMA (forward / data-grad /
// weight-grad) with the CNN epilogues fused in:
//
//   forward : rows = output pixels, k = (kh,kw,cin), B = W[cout][kh][kw][cin]
//             epilogue: +bias, ReLU, optional 2x2 max-pool *inside the registers*:
//             rows are enumerated in pool-window order (b,ph,pw,dy,dx), so the
//             4 consecutive rows a lane holds in its 16x16 MFMA accumulator are
//             exactly one pooling window -> max + argmax without any LDS trip.
//   dgrad   : rows = input pixels, k = (kh,kw,cout) over dY, B = Wt[cin][kh][kw][cout]
//             epilogue: optional un-pool (argmax scatter) + ReLU mask of the
//             layer below, writing the full-resolution gradient directly.
//   wgrad   : rows = cout, cols = (kh,kw,cin) + 1 bias column, reduction over
//             output pixels (split-K, fp32 atomics into the flat grad buffer).
//
// Replaces TF's Conv2D/Conv2DBackprop*/MaxPool*/BiasAdd*/Relu* chain
// (BASELINE.json configs 2-5).
#include "gemm_core.h"
#include "conv.h"
#include "norm.h"
#include "igemm.h"
#include <stdexcept>

namespace dtfe {

// m / d for 0 <= m < 2^24 via a float reciprocal, corrected to exact
__device__ __forceinline__ int fast_div(int m, int d, float inv_d) {
  int q = (int)((float)m * inv_d);
  const int r = m - q * d;
  q += (r >= d) - (r < 0);
  return q;
}

// decode a GEMM row into an NHWC pixel of a (RH x RW) grid
__device__ __forceinline__ void decode_row(int m, int RH, int RW, int pool_order, int& b, int& y, int& x) {
  if (pool_order) {
    const int q = m & 3, pm = m >> 2, PW = RW >> 1, PH = RH >> 1;
    const int pw = pm % PW, t = pm / PW;
    const int ph = t % PH;
    b = t / PH;
    y = 2 * ph + (q >> 1);
    x = 2 * pw + (q & 1);
  } else {
    x = m % RW;
    const int t = m / RW;
    y = t % RH;
    b = t / RH;
  }
}

// source pixel for tap (kh,kw) of row pixel (y,x).
// forward: src = (y*s - p + kh, x*s - p + kw)
// dgrad  : src = ((y + p - kh)/s, (x + p - kw)/s) when divisible
__device__ __forceinline__ bool src_pixel(const ConvGeom& g, bool transposed, int y, int x, int kh, int kw,
                                          int& sy, int& sx) {
  if (!transposed) {
    sy = y * g.stride - g.pad + kh;
    sx = x * g.stride - g.pad + kw;
    return sy >= 0 && sy < g.H && sx >= 0 && sx < g.W;
  }
  int ty = y + g.pad - kh, tx = x + g.pad - kw;
  if (ty < 0 || tx < 0) return false;
  if (g.stride > 1) {
    if ((ty % g.stride) | (tx % g.stride)) return false;
    ty /= g.stride;
    tx /= g.stride;
  }
  sy = ty;
  sx = tx;
  return sy < g.OH && sx < g.OW;
}

// A operand (KMAJ): rows = pixels of the row grid, k = (kh, kw, c) over the
// source tensor (x for forward, dY for dgrad).
//
// Every thread stages the same rows at every k-step, so each row's pixel is
// decoded once (constructor).  When the source channel count is a multiple of
// BK a k-tile never straddles two taps: (kh, kw) is wave-uniform per k-step
// and a chunk address is base + ((sy*W + sx)*C + ch) with no division.
template <int R, bool TRANS>
struct Im2colLoader {
  using Lay = LdsLayout<bf16, R, KMAJ>;
  using C = Chunks<bf16, R, KMAJ>;
  const bf16* src; ConvGeom g; int rows; int K; int r0; int SC; int RH, RW; bool cvec, fast;
  long rbase[C::NC];  // image base offset of the chunk's row (-1: row out of range)
  int ry[C::NC], rx[C::NC];
  u32x4_t regs[C::NC];

  __device__ __forceinline__ Im2colLoader(const bf16* s, const ConvGeom& g_, int r0_) : src(s), g(g_), r0(r0_) {
    if (!TRANS) { SC = g.C; RH = g.OH; RW = g.OW; }
    else { SC = g.Cout; RH = g.H; RW = g.W; }
    rows = g.B * RH * RW;
    K = g.KH * g.KW * SC;
    cvec = (SC % 8) == 0;
    fast = (SC % BK) == 0 && g.stride == 1;
    const int SH = TRANS ? g.OH : g.H, SW = TRANS ? g.OW : g.W;
#pragma unroll
    for (int c = 0; c < C::NC; ++c) {
      const int idx = threadIdx.x + c * GEMM_THREADS;
      int r, k;
      C::rk(idx, r, k);
      const int m = r0 + r;
      rbase[c] = -1;
      ry[c] = rx[c] = 0;
      if ((C::N % GEMM_THREADS == 0 || idx < C::N) && m < rows) {
        int b, y, x;
        decode_row(m, RH, RW, TRANS ? 0 : g.pool_order, b, y, x);
        rbase[c] = (long)b * SH * SW * SC;
        // stride-1 source coordinate of tap (kh,kw): forward y - p + kh ; dgrad y + p - kh
        ry[c] = TRANS ? y + g.pad : y - g.pad;
        rx[c] = TRANS ? x + g.pad : x - g.pad;
      }
    }
  }
  template <bool FAST = false>
  __device__ __forceinline__ void load(int k0) {
    const int SH = TRANS ? g.OH : g.H, SW = TRANS ? g.OW : g.W;
    if (fast) {
      const int tap = k0 / SC, ch0 = k0 - tap * SC;
      const int kh = tap / g.KW, kw = tap - kh * g.KW;
      const int dy = TRANS ? -kh : kh, dx = TRANS ? -kw : kw;
      const bool tap_ok = k0 < K;
#pragma unroll
      for (int c = 0; c < C::NC; ++c) {
        const int idx = threadIdx.x + c * GEMM_THREADS;
        int r, k;
        C::rk(idx, r, k);
        u32x4_t v = {0u, 0u, 0u, 0u};
        const int sy = ry[c] + dy, sx = rx[c] + dx;
        if (tap_ok && rbase[c] >= 0 && sy >= 0 && sy < SH && sx >= 0 && sx < SW)
          v = *reinterpret_cast<const u32x4_t*>(src + rbase[c] + ((long)sy * SW + sx) * SC + ch0 + k);
        regs[c] = v;
      }
      return;
    }
#pragma unroll
    for (int c = 0; c < C::NC; ++c) {
      const int idx = threadIdx.x + c * GEMM_THREADS;
      u32x4_t v = {0u, 0u, 0u, 0u};
      if (C::N % GEMM_THREADS == 0 || idx < C::N) {
        int r, k;
        C::rk(idx, r, k);
        const int m = r0 + r, gk = k0 + k;
        if (m < rows && gk < K) {
          int b, y, x;
          decode_row(m, RH, RW, TRANS ? 0 : g.pool_order, b, y, x);
          if (cvec) {
            const int ch = gk % SC, tap = gk / SC, kw = tap % g.KW, kh = tap / g.KW;
            int sy, sx;
            if (src_pixel(g, TRANS, y, x, kh, kw, sy, sx))
              v = *reinterpret_cast<const u32x4_t*>(src + (((long)b * SH + sy) * SW + sx) * SC + ch);
          } else {
            bf16* e = reinterpret_cast<bf16*>(&v);
#pragma unroll
            for (int i = 0; i < 8; ++i) {
              const int kk = gk + i;
              if (kk < K) {
                const int ch = kk % SC, tap = kk / SC, kw = tap % g.KW, kh = tap / g.KW;
                int sy, sx;
                if (src_pixel(g, TRANS, y, x, kh, kw, sy, sx)) e[i] = src[(((long)b * SH + sy) * SW + sx) * SC + ch];
              }
            }
          }
        }
      }
      regs[c] = v;
    }
  }
  __device__ __forceinline__ void store(bf16* lds) const { stage_store<bf16, R, KMAJ>(lds, regs); }
};

// B operand of the weight gradient (RMAJ): rows = k = (kh,kw,cin) of the
// forward conv (+ a ones row = bias column), reduction = output pixel m.
template <int R>
struct Im2colWgradLoader {
  using Lay = LdsLayout<bf16, R, RMAJ>;
  using C = Chunks<bf16, R, RMAJ>;
  const bf16* x; ConvGeom g; int Kw; int Mred; int r0; bool cvec;
  float inv_ow, inv_oh;
  int tkh[C::NC], tkw[C::NC], tch[C::NC];  // this thread's fixed k rows: tap + channel (-1: slow path)
  u32x4_t regs[C::NC];

  __device__ __forceinline__ Im2colWgradLoader(const bf16* x_, const ConvGeom& g_, int r0_) : x(x_), g(g_), r0(r0_) {
    Kw = g.KH * g.KW * g.C;
    Mred = g.B * g.OH * g.OW;
    cvec = (g.C % 8) == 0;
    inv_ow = 1.f / (float)g.OW;
    inv_oh = 1.f / (float)g.OH;
#pragma unroll
    for (int c = 0; c < C::NC; ++c) {
      const int idx = threadIdx.x + c * GEMM_THREADS;
      int r, k;
      C::rk(idx, r, k);
      const int gr = r0 + r;
      tch[c] = -1;
      tkh[c] = tkw[c] = 0;
      if (cvec && gr + 8 <= Kw) {
        const int tap = gr / g.C;
        tch[c] = gr - tap * g.C;
        tkh[c] = tap / g.KW;
        tkw[c] = tap - tkh[c] * g.KW;
      }
    }
  }
  template <bool FAST = false>
  __device__ __forceinline__ void load(int k0) {
#pragma unroll
    for (int c = 0; c < C::NC; ++c) {
      const int idx = threadIdx.x + c * GEMM_THREADS;
      u32x4_t v = {0u, 0u, 0u, 0u};
      if (C::N % GEMM_THREADS == 0 || idx < C::N) {
        int r, k;
        C::rk(idx, r, k);
        const int m = k0 + k, gr = r0 + r;
        if (m < Mred) {
          // m -> (b, y, x) without integer division
          const int q1 = fast_div(m, g.OW, inv_ow);
          const int xx = m - q1 * g.OW;
          const int b = fast_div(q1, g.OH, inv_oh);
          const int y = q1 - b * g.OH;
          bf16* e = reinterpret_cast<bf16*>(&v);
          if (tch[c] >= 0) {
            const int sy = y * g.stride - g.pad + tkh[c], sx = xx * g.stride - g.pad + tkw[c];
            if (sy >= 0 && sy < g.H && sx >= 0 && sx < g.W)
              v = *reinterpret_cast<const u32x4_t*>(x + (((long)b * g.H + sy) * g.W + sx) * g.C + tch[c]);
          } else {
#pragma unroll
            for (int i = 0; i < 8; ++i) {
              const int kk = gr + i;
              if (kk < Kw) {
                const int ch = kk % g.C, tap = kk / g.C, kw = tap % g.KW, kh = tap / g.KW;
                int sy, sx;
                if (src_pixel(g, false, y, xx, kh, kw, sy, sx)) e[i] = x[(((long)b * g.H + sy) * g.W + sx) * g.C + ch];
              } else if (kk == Kw) {
                e[i] = 0x3f80;  // bias column
              }
            }
          }
        }
      }
      regs[c] = v;
    }
  }
  __device__ __forceinline__ void store(bf16* lds) const { stage_store<bf16, R, RMAJ>(lds, regs); }
};

// ------------------------------------------------------------------ forward
template <typename Cfg>
__global__ __launch_bounds__(GEMM_THREADS) void conv_fwd_kernel(ConvFwdArgs a) {
  using LA = Im2colLoader<Cfg::BM, false>;
  using LB = DenseLoader<bf16, Cfg::BN, KMAJ>;
  __shared__ __attribute__((aligned(16))) bf16 smem[SmemSize<bf16, Cfg, LA, LB>::ELEMS];
  const ConvGeom& g = a.g;
  const int M = g.B * g.OH * g.OW, N = g.Cout, K = g.KH * g.KW * g.C;
  const int tiles_m = (M + Cfg::BM - 1) / Cfg::BM, tiles_n = (N + Cfg::BN - 1) / Cfg::BN;
  int tm, tn;
  tile_coords(tiles_m, tiles_n, tm, tn);
  const int m_base = tm * Cfg::BM, n_base = tn * Cfg::BN;
  LA la(a.x, g, m_base);
  LB lb(a.w, K, N, K, n_base);
  f32x4_t acc[Cfg::TM][Cfg::TN];
  gemm_mainloop<bf16, Cfg, KMAJ, KMAJ>(la, lb, 0, K, smem, acc);

  for_each_quad<Cfg>(m_base, n_base, acc, [&](int row0, int col, f32x4_t v) {
    if (col >= N || row0 >= M) return;  // M is a multiple of 4 in pool mode
    const float bias = a.bias ? a.bias[col] : 0.f;
    if (g.pool_order) {
      int am = 0;
      float mx = v[0];
#pragma unroll
      for (int j = 1; j < 4; ++j) if (v[j] > mx) { mx = v[j]; am = j; }
      const float y = apply_act(mx + bias, a.act);  // act is monotone: pool(act(z)) == act(pool(z))
      const long o = (long)(row0 >> 2) * N + col;
      a.y[o] = f2bf(y);
      if (a.argmax) a.argmax[o] = (uint8_t)am;
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (row0 + j < M) a.y[(long)(row0 + j) * N + col] = f2bf(apply_act(v[j] + bias, a.act));
      }
    }
  });
}

// ------------------------------------------------------------------- dgrad
template <typename Cfg>
__global__ __launch_bounds__(GEMM_THREADS) void conv_dgrad_kernel(ConvDgradArgs a) {
  using LA = Im2colLoader<Cfg::BM, true>;
  using LB = DenseLoader<bf16, Cfg::BN, KMAJ>;
  __shared__ __attribute__((aligned(16))) bf16 smem[SmemSize<bf16, Cfg, LA, LB>::ELEMS];
  const ConvGeom& g = a.g;
  const int M = g.B * g.H * g.W, N = g.C, K = g.KH * g.KW * g.Cout;
  const int tiles_m = (M + Cfg::BM - 1) / Cfg::BM, tiles_n = (N + Cfg::BN - 1) / Cfg::BN;
  int tm, tn;
  tile_coords(tiles_m, tiles_n, tm, tn);
  const int m_base = tm * Cfg::BM, n_base = tn * Cfg::BN;
  LA la(a.dy, g, m_base);
  LB lb(a.wt, K, N, K, n_base);
  f32x4_t acc[Cfg::TM][Cfg::TN];
  gemm_mainloop<bf16, Cfg, KMAJ, KMAJ>(la, lb, 0, K, smem, acc);

  for_each_quad<Cfg>(m_base, n_base, acc, [&](int row0, int col, f32x4_t v) {
    if (col >= N) return;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int m = row0 + j;
      if (m >= M) continue;
      const long pidx = (long)m * N + col;
      if (a.unpool) unpool_store(a.up, pidx, v[j], a.dx);
      else if (a.relu_mask) a.dx[pidx] = f2bf(bf2f(a.relu_mask[pidx]) > 0.f ? v[j] : 0.f);
      else a.dx[pidx] = f2bf(v[j]);
    }
  });
}

// ------------------------------------------------------------------- wgrad
template <typename Cfg>
__global__ __launch_bounds__(GEMM_THREADS) void conv_wgrad_kernel(ConvWgradArgs a) {
  using LA = DenseLoader<bf16, Cfg::BM, RMAJ>;  // dZ[m][cout]
  using LB = Im2colWgradLoader<Cfg::BN>;
  __shared__ __attribute__((aligned(16))) bf16 smem[SmemSize<bf16, Cfg, LA, LB>::ELEMS];
  const ConvGeom& g = a.g;
  const int M = g.Cout, Kw = g.KH * g.KW * g.C, N = Kw + (a.db ? 1 : 0), Kred = g.B * g.OH * g.OW;
  const int tiles_m = (M + Cfg::BM - 1) / Cfg::BM, tiles_n = (N + Cfg::BN - 1) / Cfg::BN;
  int tm, tn;
  tile_coords(tiles_m, tiles_n, tm, tn);
  const int m_base = tm * Cfg::BM, n_base = tn * Cfg::BN;
  const int k_begin = blockIdx.z * a.k_chunk;
  const int k_end = min(Kred, k_begin + a.k_chunk);
  LA la(a.dz, M, M, Kred, m_base);
  LB lb(a.x, g, n_base);
  f32x4_t acc[Cfg::TM][Cfg::TN];
  gemm_mainloop<bf16, Cfg, RMAJ, RMAJ>(la, lb, k_begin, k_end, smem, acc);

  for_each_quad<Cfg>(m_base, n_base, acc, [&](int row0, int col, f32x4_t v) {
    if (col > Kw || (col == Kw && !a.db)) return;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int row = row0 + j;
      if (row >= M) continue;
      if (col < Kw) atomicAdd(a.dw + (long)row * Kw + col, v[j] * a.scale);
      else atomicAdd(a.db + row, v[j] * a.scale);
    }
  });
}

// ------------------------------------------------------------------ launch
template <typename Cfg> static int tiles_of(int M, int N) {
  return ((M + Cfg::BM - 1) / Cfg::BM) * ((N + Cfg::BN - 1) / Cfg::BN);
}

// Tile policy for the skinny-N convolutions (N = Cout or C <= 64, M = pixels):
// tall 256-row tiles (4 waves stacked along M, each wave 64 x N) give 8-16
// MFMAs per wave per k-step and still >= 1 workgroup per CU once M >= 64K.
template <template <typename> class KERN, typename ARGS>
static void launch_skinny(const ARGS& a, int M, int N, hipStream_t s) {
  const bool tall = M >= 256 * 256;
  if (N <= 32) {
    if (tall) {
      using Cfg = TileCfg<bf16, 256, 32, 4, 1>;
      hipLaunchKernelGGL(KERN<Cfg>::fn, dim3(tiles_of<Cfg>(M, N)), dim3(GEMM_THREADS), 0, s, a);
    } else {
      using Cfg = TileCfg<bf16, 128, 32, 4, 1>;
      hipLaunchKernelGGL(KERN<Cfg>::fn, dim3(tiles_of<Cfg>(M, N)), dim3(GEMM_THREADS), 0, s, a);
    }
  } else if (N <= 64) {
    if (tall) {
      using Cfg = TileCfg<bf16, 256, 64, 4, 1>;
      hipLaunchKernelGGL(KERN<Cfg>::fn, dim3(tiles_of<Cfg>(M, N)), dim3(GEMM_THREADS), 0, s, a);
    } else {
      using Cfg = TileCfg<bf16, 128, 64, 2, 2>;
      hipLaunchKernelGGL(KERN<Cfg>::fn, dim3(tiles_of<Cfg>(M, N)), dim3(GEMM_THREADS), 0, s, a);
    }
  } else {
    using Cfg = TileCfg<bf16, 128, 128, 2, 2>;
    hipLaunchKernelGGL(KERN<Cfg>::fn, dim3(tiles_of<Cfg>(M, N)), dim3(GEMM_THREADS), 0, s, a);
  }
}

template <typename Cfg> struct FwdK { static constexpr auto fn = conv_fwd_kernel<Cfg>; };
template <typename Cfg> struct DgradK { static constexpr auto fn = conv_dgrad_kernel<Cfg>; };

// BatchNorm statistics of a conv output by the separate pass (paths without fused partials)
static void bn_stats_of(const ConvFwdArgs& a, hipStream_t s) {
  if (!a.bn_stats) return;
  if (a.g.pool_order) throw std::runtime_error("conv_fwd: bn_stats with a fused pool");
  BnArgs b{};
  b.R = (long)a.g.B * a.g.OH * a.g.OW;
  b.C = a.g.Cout;
  b.x = a.y;
  b.stats = a.bn_stats;
  launch_bn_stats(b, s);
}

void launch_conv_fwd(const ConvFwdArgs& a, hipStream_t s) {
  bool stem_stats = false;
  if (launch_stem_fwd(a, s, &stem_stats)) {  // ImageNet 7x7/2 stem (+ BN partials in its epilogue)
    if (!stem_stats) bn_stats_of(a, s);
    return;
  }
  bool fused = false;
  if (launch_igemm_fwd(a, s, &fused)) {  // wide layers: DMA-staged 64-deep k-tiles (+ BN partials)
    if (!fused) bn_stats_of(a, s);
    return;
  }
  const ConvGeom& g = a.g;
  if (g.pool_order && ((g.OH | g.OW) & 1)) throw std::runtime_error("conv_fwd: pool needs even output dims");
  launch_skinny<FwdK>(a, g.B * g.OH * g.OW, g.Cout, s);
  bn_stats_of(a, s);
}

void launch_dgrad_bn_bwd_stats(const ConvDgradArgs& a, hipStream_t s) {
  BnArgs b{};
  b.R = (long)a.g.B * a.g.H * a.g.W;
  b.C = a.g.C;
  b.x = a.bnb_x; b.y = a.bnb_y; b.dy = a.dx; b.ymask = a.bnb_ymask;
  b.stats = a.bnb_stats;
  b.gamma = a.bnb_gamma; b.beta = a.bnb_beta;
  b.mean = const_cast<float*>(a.bnb_mean); b.invstd = const_cast<float*>(a.bnb_invstd);
  b.act = a.bnb_act;
  launch_bn_bwd_stats(b, s);
}

void launch_conv_dgrad(const ConvDgradArgs& a, hipStream_t s) {
  if (launch_igemm_dgrad(a, s)) return;
  if (a.accumulate) throw std::runtime_error("conv_dgrad: accumulate needs the implicit-GEMM path (C, Cout % 64 == 0)");
  const ConvGeom& g = a.g;
  launch_skinny<DgradK>(a, g.B * g.H * g.W, g.C, s);
  if (a.bnb_stats) launch_dgrad_bn_bwd_stats(a, s);
}

template <typename Cfg>
static void wgrad_launch(const ConvWgradArgs& a0, int target_blocks, hipStream_t s) {
  ConvWgradArgs a = a0;
  const ConvGeom& g = a.g;
  const int M = g.Cout, N = g.KH * g.KW * g.C + (a.db ? 1 : 0), Kred = g.B * g.OH * g.OW;
  const int tiles = tiles_of<Cfg>(M, N);
  int splits = (target_blocks + tiles - 1) / tiles;
  int chunk = (Kred + splits - 1) / splits;
  chunk = ((chunk + BK - 1) / BK) * BK;
  if (chunk < 4 * BK) chunk = 4 * BK;
  splits = (Kred + chunk - 1) / chunk;
  a.k_chunk = chunk;
  hipLaunchKernelGGL(conv_wgrad_kernel<Cfg>, dim3(tiles, 1, splits), dim3(GEMM_THREADS), 0, s, a);
}

void launch_conv_wgrad(const ConvWgradArgs& a, hipStream_t s) {
  if (launch_stem_wgrad(a, s, true)) return;
  if (launch_igemm_wgrad(a, s)) return;
  const ConvGeom& g = a.g;
  const int M = g.Cout, N = g.KH * g.KW * g.C + (a.db ? 1 : 0);
  const int target = 1024;  // 4 workgroups per CU
  if (M <= 32 && N <= 32) wgrad_launch<TileCfg<bf16, 32, 32, 2, 2>>(a, target, s);
  else if (M <= 64) wgrad_launch<TileCfg<bf16, 64, 128, 2, 2>>(a, target, s);
  else wgrad_launch<TileCfg<bf16, 128, 128, 2, 2>>(a, target, s);
}

}  // namespace dtfe
