// Exact-fp32 NHWC convolution (the reference's precision, `--dtype fp32`): forward (+bias, ReLU,
// fused 2x2 max-pool + argmax), data gradient (+ReLU mask of a pooled consumer), weight gradient
// (+bias gradient), plus the two small data movers the fp32 CNN step needs (2x2 un-pool of a
// pooled gradient, [O][T][C] -> [C][T][O] weight transpose for the data gradient).
//
// The matrix work runs on v_mfma_f32_16x16x4_f32 through the generic LDS-tiled engine of
// gemm_core.h (T = float: 16-B chunks of 4 k, KMAJ images [rows][32 + 4]): the same fp32-in /
// fp32-accumulate arithmetic as an fmaf chain, so the step matches fp32 autograd to rounding.
// The im2col operands are gathered per 16-B chunk (4 consecutive channels of one tap) when the
// channel count is a multiple of 4, element by element otherwise (the 1-channel MNIST input).
//
// Replaces Conv2D / Conv2DBackpropInput / Conv2DBackpropFilter / MaxPool(+grad) / BiasAdd(+grad)
// / Relu(+grad) of the MNIST CNN at fp32 (TensorFlow-Examples convolutional_network, the notebook
// family of ENC:14; fp32 as every reference script: GAN:122-135, LSTM:83-97).
#include "gemm_core.h"
#include "conv.h"
#include "conv_f32.h"
#include "imgconv.h"  // launch_partials_reduce

#include <algorithm>

namespace dtfe {

namespace {

__device__ __forceinline__ int fdiv(int m, int d, float inv_d) {
  int q = (int)((float)m * inv_d);
  const int r = m - q * d;
  q += (r >= d) - (r < 0);
  return q;
}

// row m of the output grid -> (b, y, x); pool order enumerates 2x2 windows (b, ph, pw, dy, dx)
__device__ __forceinline__ void f32_row(int m, int RH, int RW, int pool_order, int& b, int& y, int& x) {
  if (pool_order) {
    const int q = m & 3, pm = m >> 2, PW = RW >> 1, PH = RH >> 1;
    const int pw = pm % PW, t = pm / PW;
    y = 2 * (t % PH) + (q >> 1);
    x = 2 * pw + (q & 1);
    b = t / PH;
  } else {
    x = m % RW;
    const int t = m / RW;
    y = t % RH;
    b = t / RH;
  }
}

// A operand (KMAJ): rows = pixels of the row grid, k = (kh, kw, c) of the source.
// TRANS (data gradient): source = dY, stride-1 flipped taps: src = (y + p - kh, x + p - kw).
template <int R, bool TRANS>
struct Im2colF32 {
  using Lay = LdsLayout<float, R, KMAJ>;
  using C = Chunks<float, R, KMAJ>;
  const float* src; ConvGeom g; int rows, K, SC, SH, SW;
  float inv_sc, inv_kw;  // (reciprocal divisions: two runtime integer divisions per chunk and k-step otherwise)
  int rb[C::NC], ry[C::NC], rx[C::NC];  // per chunk: batch (-1: out of range), tap-0 source coords
  u32x4_t regs[C::NC];

  __device__ __forceinline__ Im2colF32(const float* s, const ConvGeom& g_, int r0) : src(s), g(g_) {
    const int RH = TRANS ? g.H : g.OH, RW = TRANS ? g.W : g.OW;
    SC = TRANS ? g.Cout : g.C;
    SH = TRANS ? g.OH : g.H;
    SW = TRANS ? g.OW : g.W;
    rows = g.B * RH * RW;
    K = g.KH * g.KW * SC;
    inv_sc = 1.f / (float)SC;
    inv_kw = 1.f / (float)g.KW;
#pragma unroll
    for (int c = 0; c < C::NC; ++c) {
      int r, k;
      C::rk(threadIdx.x + c * GEMM_THREADS, r, k);
      const int m = r0 + r;
      rb[c] = -1;
      ry[c] = rx[c] = 0;
      if ((C::N % GEMM_THREADS == 0 || threadIdx.x + c * GEMM_THREADS < C::N) && m < rows) {
        int b, y, x;
        f32_row(m, RH, RW, TRANS ? 0 : g.pool_order, b, y, x);
        rb[c] = b;
        ry[c] = TRANS ? y + g.pad : y * g.stride - g.pad;
        rx[c] = TRANS ? x + g.pad : x * g.stride - g.pad;
      }
    }
  }
  __device__ __forceinline__ float at(int c, int gk) const {
    const int tap = gk / SC, ch = gk - tap * SC, kh = tap / g.KW, kw = tap - kh * g.KW;
    const int sy = TRANS ? ry[c] - kh : ry[c] + kh, sx = TRANS ? rx[c] - kw : rx[c] + kw;
    if (sy < 0 || sy >= SH || sx < 0 || sx >= SW) return 0.f;
    return src[(((long)rb[c] * SH + sy) * SW + sx) * SC + ch];
  }
  template <bool FAST = false>
  __device__ __forceinline__ void load(int k0) {
#pragma unroll
    for (int c = 0; c < C::NC; ++c) {
      int r, k;
      C::rk(threadIdx.x + c * GEMM_THREADS, r, k);
      const int gk = k0 + k;
      f32x4_t v = {0.f, 0.f, 0.f, 0.f};
      if (rb[c] >= 0 && gk < K) {
        if ((SC & 3) == 0) {  // 4 channels of one tap: one 16-B load
          const int tap = fdiv(gk, SC, inv_sc), ch = gk - tap * SC, kh = fdiv(tap, g.KW, inv_kw), kw = tap - kh * g.KW;
          const int sy = TRANS ? ry[c] - kh : ry[c] + kh, sx = TRANS ? rx[c] - kw : rx[c] + kw;
          if (sy >= 0 && sy < SH && sx >= 0 && sx < SW)
            v = *reinterpret_cast<const f32x4_t*>(src + (((long)rb[c] * SH + sy) * SW + sx) * SC + ch);
        } else {
#pragma unroll
          for (int i = 0; i < 4; ++i) v[i] = gk + i < K ? at(c, gk + i) : 0.f;
        }
      }
      regs[c] = __builtin_bit_cast(u32x4_t, v);
    }
  }
  __device__ __forceinline__ void store(float* lds) const { stage_store<float, R, KMAJ>(lds, regs); }
};

// B operand of the weight gradient (RMAJ, transposed while staging): rows = k = (kh, kw, c) of the
// forward conv + one ones row (the bias column), reduction = output pixel m.  A thread's chunk rows
// (4 consecutive k) are the same at every k-step (Chunks<RMAJ>: only the pixel moves), so their
// (kh, kw, c) decomposition is done once here; a load is then two reciprocal divisions of the pixel
// index and, when C % 4 == 0, ONE 16-B load of 4 channels of one tap (per-element loads with four
// runtime integer divisions each had the conv2 weight gradient at ~26 TFLOP/s, 800 us per step).
template <int R>
struct Im2colWgradF32 {
  using Lay = LdsLayout<float, R, RMAJ>;
  using C = Chunks<float, R, RMAJ>;
  const float* x; ConvGeom g; int Mred;
  float inv_ow, inv_oh;
  static_assert(GEMM_THREADS % (R / 4) == 0, "a thread's chunks must share their rows");
  int kh[4], kw[4], off[4];  // per chunk row: tap coordinates and channel offset; kh = -1: zero, -2: ones
  bool vec;                  // the 4 rows are 4 channels of one tap (C % 4 == 0)
  u32x4_t regs[C::NC];

  __device__ __forceinline__ Im2colWgradF32(const float* x_, const ConvGeom& g_, int r0) : x(x_), g(g_) {
    const int Kw = g.KH * g.KW * g.C;
    Mred = g.B * g.OH * g.OW;
    inv_ow = 1.f / (float)g.OW;
    inv_oh = 1.f / (float)g.OH;
    int r, k;
    C::rk(threadIdx.x, r, k);  // (the same rows for every chunk of this thread)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int kk = r0 + r + i;
      kh[i] = kk == Kw ? -2 : -1;
      kw[i] = off[i] = 0;
      if (kk < Kw) {
        const int tap = kk / g.C;
        kh[i] = tap / g.KW;
        kw[i] = tap - kh[i] * g.KW;
        off[i] = kk - tap * g.C;
      }
    }
    vec = (g.C & 3) == 0 && kh[0] >= 0 && kh[3] >= 0;
  }
  template <bool FAST = false>
  __device__ __forceinline__ void load(int k0) {
#pragma unroll
    for (int c = 0; c < C::NC; ++c) {
      f32x4_t v = {0.f, 0.f, 0.f, 0.f};
      const int idx = threadIdx.x + c * GEMM_THREADS;
      if (C::N % GEMM_THREADS == 0 || idx < C::N) {
        int r, k;
        C::rk(idx, r, k);
        const int m = k0 + k;
        if (m < Mred) {
          const int q1 = fdiv(m, g.OW, inv_ow);
          const int ox = m - q1 * g.OW;
          const int b = fdiv(q1, g.OH, inv_oh);
          const int oy = q1 - b * g.OH;
          const int y0 = oy * g.stride - g.pad, x0 = ox * g.stride - g.pad;
          const float* xb = x + (long)b * g.H * g.W * g.C;
          if (vec) {
            const int sy = y0 + kh[0], sx = x0 + kw[0];
            if (sy >= 0 && sy < g.H && sx >= 0 && sx < g.W)
              v = *reinterpret_cast<const f32x4_t*>(xb + ((long)sy * g.W + sx) * g.C + off[0]);
          } else {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const int sy = y0 + kh[i], sx = x0 + kw[i];
              if (kh[i] == -2) v[i] = 1.f;  // bias column
              else if (kh[i] >= 0 && sy >= 0 && sy < g.H && sx >= 0 && sx < g.W)
                v[i] = xb[((long)sy * g.W + sx) * g.C + off[i]];
            }
          }
        }
      }
      regs[c] = __builtin_bit_cast(u32x4_t, v);
    }
  }
  __device__ __forceinline__ void store(float* lds) const { stage_store<float, R, RMAJ>(lds, regs); }
};

template <typename Cfg>
__global__ __launch_bounds__(GEMM_THREADS) void conv_fwd_f32_kernel(ConvF32Args a) {
  using LA = Im2colF32<Cfg::BM, false>;
  using LB = DenseLoader<float, Cfg::BN, KMAJ>;
  __shared__ __attribute__((aligned(16))) float smem[SmemSize<float, Cfg, LA, LB>::ELEMS];
  const ConvGeom& g = a.g;
  const int M = g.B * g.OH * g.OW, N = g.Cout, K = g.KH * g.KW * g.C;
  int tm, tn;
  tile_coords((M + Cfg::BM - 1) / Cfg::BM, (N + Cfg::BN - 1) / Cfg::BN, tm, tn);
  const int m_base = tm * Cfg::BM, n_base = tn * Cfg::BN;
  LA la(a.src, g, m_base);
  LB lb(a.w, K, N, K, n_base);
  f32x4_t acc[Cfg::TM][Cfg::TN];
  gemm_mainloop<float, Cfg, KMAJ, KMAJ>(la, lb, 0, K, smem, acc);
  for_each_quad<Cfg>(m_base, n_base, acc, [&](int row0, int col, f32x4_t v) {
    if (col >= N || row0 >= M) return;
    const float bias = a.bias ? a.bias[col] : 0.f;
    if (g.pool_order) {  // the 4 rows of a lane are one 2x2 window; first maximum wins (torch / TF)
      int am = 0;
      float mx = v[0];
#pragma unroll
      for (int j = 1; j < 4; ++j)
        if (v[j] > mx) { mx = v[j]; am = j; }
      const long o = (long)(row0 >> 2) * N + col;
      a.out[o] = apply_act(mx + bias, a.act);  // act is monotone: pool(act(z)) == act(pool(z))
      if (a.argmax) a.argmax[o] = (uint8_t)am;
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (row0 + j < M) a.out[(long)(row0 + j) * N + col] = apply_act(v[j] + bias, a.act);
    }
  });
}

template <typename Cfg>
__global__ __launch_bounds__(GEMM_THREADS) void conv_dgrad_f32_kernel(ConvF32Args a) {
  using LA = Im2colF32<Cfg::BM, true>;
  using LB = DenseLoader<float, Cfg::BN, KMAJ>;  // wt [C][KH][KW][Cout]
  __shared__ __attribute__((aligned(16))) float smem[SmemSize<float, Cfg, LA, LB>::ELEMS];
  const ConvGeom& g = a.g;
  const int M = g.B * g.H * g.W, N = g.C, K = g.KH * g.KW * g.Cout;
  int tm, tn;
  tile_coords((M + Cfg::BM - 1) / Cfg::BM, (N + Cfg::BN - 1) / Cfg::BN, tm, tn);
  const int m_base = tm * Cfg::BM, n_base = tn * Cfg::BN;
  LA la(a.src, g, m_base);
  LB lb(a.w, K, N, K, n_base);
  f32x4_t acc[Cfg::TM][Cfg::TN];
  gemm_mainloop<float, Cfg, KMAJ, KMAJ>(la, lb, 0, K, smem, acc);
  for_each_quad<Cfg>(m_base, n_base, acc, [&](int row0, int col, f32x4_t v) {
    if (col >= N) return;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const long o = (long)(row0 + j) * N + col;
      if (row0 + j < M) a.out[o] = (!a.relu_mask || a.relu_mask[o] > 0.f) ? v[j] : 0.f;
    }
  });
}

template <typename Cfg>
__global__ __launch_bounds__(GEMM_THREADS) void conv_wgrad_f32_kernel(ConvF32Args a) {
  using LA = DenseLoader<float, Cfg::BM, RMAJ>;  // dZ[m][cout]
  using LB = Im2colWgradF32<Cfg::BN>;
  __shared__ __attribute__((aligned(16))) float smem[SmemSize<float, Cfg, LA, LB>::ELEMS];
  const ConvGeom& g = a.g;
  const int M = g.Cout, Kw = g.KH * g.KW * g.C, N = Kw + (a.db ? 1 : 0), Kred = g.B * g.OH * g.OW;
  int tm, tn;
  tile_coords((M + Cfg::BM - 1) / Cfg::BM, (N + Cfg::BN - 1) / Cfg::BN, tm, tn);
  const int m_base = tm * Cfg::BM, n_base = tn * Cfg::BN;
  const int k_begin = blockIdx.z * a.k_chunk, k_end = min(Kred, k_begin + a.k_chunk);
  LA la(a.src, M, M, Kred, m_base);
  LB lb(a.x, g, n_base);
  f32x4_t acc[Cfg::TM][Cfg::TN];
  gemm_mainloop<float, Cfg, RMAJ, RMAJ>(la, lb, k_begin, k_end, smem, acc);
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

template <typename Cfg> int ntiles(int M, int N) { return ((M + Cfg::BM - 1) / Cfg::BM) * ((N + Cfg::BN - 1) / Cfg::BN); }

// one thread per pooled element: route g to its argmax position of the 2x2 window, zeros elsewhere
__global__ __launch_bounds__(256) void unpool_f32_kernel(const float* __restrict__ g, const uint8_t* __restrict__ am,
                                                         float* __restrict__ out, int PH, int PW, int C, long n) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int c = (int)(i % C);
  long t = i / C;
  const int pw = (int)(t % PW);
  t /= PW;
  const int ph = (int)(t % PH);
  const long b = t / PH;
  const int q0 = am[i];
  const float v = g[i];
#pragma unroll
  for (int q = 0; q < 4; ++q)
    out[((b * 2 * PH + 2 * ph + (q >> 1)) * 2 * PW + 2 * pw + (q & 1)) * C + c] = q == q0 ? v : 0.f;
}

// out[c][t][o] = in[o][t][c]
__global__ __launch_bounds__(256) void transpose_taps_f32_kernel(const float* __restrict__ in, float* __restrict__ out,
                                                                 int O, int T, int C) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)O * T * C) return;
  const int c = (int)(i % C);
  const long r = i / C;
  const int t = (int)(r % T), o = (int)(r / T);
  out[((long)c * T + t) * O + o] = in[i];
}

// ------------------------------------------------------------------ the 1-channel input layer
// MNIST conv1 (C = 1, 32 output channels, KSxKS SAME, stride 1, 2x2 max-pool) at fp32.  With one input
// channel the GEMM view has K = KS*KS = 25 (one and a half 16-deep MFMA steps of padding, every A
// element gathered on its own), so the generic im2col kernels spent 74 us (forward) and 174 us
// (weight gradient over the materialised 103 MB un-pooled gradient) on 1.3 GFLOP.  These kernels
// work on VALU fmaf chains over an LDS-staged image instead:
//   forward   thread = (channel n, pooled pixel q): the 6x6 input window of its 2x2 pool window
//             (broadcast LDS reads: the 32 lanes of a q read one window) x 25 register weights,
//             the four outputs as packed fp32 FMAs, first-max argmax, bias + act - in the same k
//             order as the generic kernel's fmaf chain;
//   wgrad     thread = (channel n, tap row kh, q parity): for every pooled gradient only the argmax
//             pixel of its window is non-zero, so dW[n][kh][kw] += dP[q][n] * x[pixel(q, n) + tap]
//             over the pooled positions (a quarter of the dense products, no un-pooled tensor),
//             per-workgroup partial slabs summed by partials_reduce in a fixed order (no float
//             atomics: the fp32 step is run-to-run deterministic).
constexpr int C1F_N = 32, C1F_LP = 36;  // channels; LDS plane pitch (W + KS - 1 <= 36)
typedef float f32x2v __attribute__((ext_vector_type(2)));

template <int KS>
__global__ __launch_bounds__(256) void conv1_fwd_pool_f32_kernel(ConvF32Args a) {
  constexpr int T = KS * KS, WIN = KS + 1;
  __shared__ float xs[C1F_LP * C1F_LP];
  const ConvGeom& g = a.g;
  const int H = g.H, W = g.W, PH = H >> 1, PW = W >> 1, NQ = PH * PW, HW = H * W;
  const int tid = threadIdx.x, n = tid & 31, qi = tid >> 5;
  float wr[T];
#pragma unroll
  for (int t = 0; t < T; ++t) wr[t] = a.w[n * T + t];
  const float bias = a.bias ? a.bias[n] : 0.f;
  for (int i = tid; i < C1F_LP * C1F_LP; i += 256) xs[i] = 0.f;
  // the image's pixels, 4 per thread (H*W <= 1024): prefetched one image ahead
  float xv[4];
  auto load = [&](long b) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int i = tid + j * 256;
      xv[j] = i < HW ? a.src[b * HW + i] : 0.f;
    }
  };
  long b = blockIdx.x;
  if (b < g.B) load(b);
  __syncthreads();
  for (; b < g.B; b += gridDim.x) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int i = tid + j * 256;
      if (i < HW) {
        const int y = i / W, x = i - y * W;
        xs[(y + KS / 2) * C1F_LP + x + KS / 2] = xv[j];
      }
    }
    __syncthreads();
    if (b + gridDim.x < g.B) load(b + gridDim.x);
    for (int q = qi; q < NQ; q += 8) {
      const int py = q / PW, px = q - py * PW;
      const float* base = xs + (2 * py) * C1F_LP + 2 * px;
      float win[WIN][WIN];
#pragma unroll
      for (int r = 0; r < WIN; ++r)
#pragma unroll
        for (int c = 0; c < WIN; ++c) win[r][c] = base[r * C1F_LP + c];
      f32x2v z0 = {0.f, 0.f}, z1 = {0.f, 0.f};  // (dy = 0: dx 0, 1), (dy = 1: dx 0, 1)
#pragma unroll
      for (int kh = 0; kh < KS; ++kh)
#pragma unroll
        for (int kw = 0; kw < KS; ++kw) {
          const float w = wr[kh * KS + kw];
          z0 = __builtin_elementwise_fma(f32x2v{w, w}, f32x2v{win[kh][kw], win[kh][kw + 1]}, z0);
          z1 = __builtin_elementwise_fma(f32x2v{w, w}, f32x2v{win[kh + 1][kw], win[kh + 1][kw + 1]}, z1);
        }
      const float z[4] = {z0[0], z0[1], z1[0], z1[1]};
      int am = 0;
      float mx = z[0];
#pragma unroll
      for (int j = 1; j < 4; ++j)
        if (z[j] > mx) { mx = z[j]; am = j; }
      const long o = ((b * PH + py) * PW + px) * C1F_N + n;
      a.out[o] = apply_act(mx + bias, a.act);  // act is monotone: pool(act(z)) == act(pool(z))
      if (a.argmax) a.argmax[o] = (uint8_t)am;
    }
    __syncthreads();
  }
}

// dP [B][PH][PW][32] fp32 (the ReLU mask already applied), argmax bytes of the same layout, x [B][H][W]
// -> ws[blockIdx][32*T + 32] = (dW[n][t], db[n]) partial sums over the workgroup's images
template <int KS>
__global__ __launch_bounds__(320) void conv1_wgrad_pooled_f32_kernel(const float* __restrict__ dp,
                                                                     const uint8_t* __restrict__ am,
                                                                     const float* __restrict__ x, float* ws, int B,
                                                                     int H, int W) {
  constexpr int T = KS * KS, TH = 320, LEN = C1F_N * T + C1F_N;
  static_assert(KS <= 5, "the 320-thread mapping covers 5 tap rows x 32 channels x 2 q parities");
  __shared__ float xs[C1F_LP * C1F_LP];
  __shared__ __attribute__((aligned(16))) float gs[32 * 32 * C1F_N / 4];  // pooled gradient image (<= 16x16)
  __shared__ __attribute__((aligned(16))) uint8_t as[32 * 32 * C1F_N / 4];
  __shared__ float red[KS * C1F_N * KS + C1F_N];
  const int PH = H >> 1, PW = W >> 1, NQ = PH * PW, HW = H * W, NG = NQ * C1F_N;
  const int tid = threadIdx.x, n = tid & 31, kh = (tid >> 5) % 5, qh = tid / 160;
  const bool act_t = kh < KS;
  float acc[KS], dbacc = 0.f;
#pragma unroll
  for (int j = 0; j < KS; ++j) acc[j] = 0.f;
  for (int i = tid; i < C1F_LP * C1F_LP; i += TH) xs[i] = 0.f;
  // per image: NG / 4 16-B gradient chunks, NG / 16 16-B argmax chunks, HW pixels; prefetched one
  // image ahead in registers (NG <= 8192: 7 gradient chunks, 2 argmax chunks, 4 pixels per thread)
  constexpr int GC = (32 * 32 * C1F_N / 4 / 4 + TH - 1) / TH, AC = (32 * 32 * C1F_N / 4 / 16 + TH - 1) / TH;
  f32x4_t gv[GC];
  u32x4_t av[AC];
  float xv[4];
  auto load = [&](long b) {
#pragma unroll
    for (int j = 0; j < GC; ++j) {
      const int i = tid + j * TH;
      if (i < NG / 4) gv[j] = *reinterpret_cast<const f32x4_t*>(dp + b * NG + i * 4);
    }
#pragma unroll
    for (int j = 0; j < AC; ++j) {
      const int i = tid + j * TH;
      if (i < NG / 16) av[j] = *reinterpret_cast<const u32x4_t*>(am + b * NG + i * 16);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int i = tid + j * TH;
      xv[j] = i < HW ? x[b * HW + i] : 0.f;
    }
  };
  long b = blockIdx.x;
  if (b < B) load(b);
  __syncthreads();
  for (; b < B; b += gridDim.x) {
#pragma unroll
    for (int j = 0; j < GC; ++j) {
      const int i = tid + j * TH;
      if (i < NG / 4) reinterpret_cast<f32x4_t*>(gs)[i] = gv[j];
    }
#pragma unroll
    for (int j = 0; j < AC; ++j) {
      const int i = tid + j * TH;
      if (i < NG / 16) reinterpret_cast<u32x4_t*>(as)[i] = av[j];
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int i = tid + j * TH;
      if (i < HW) {
        const int y = i / W, xx = i - y * W;
        xs[(y + KS / 2) * C1F_LP + xx + KS / 2] = xv[j];
      }
    }
    __syncthreads();
    if (b + gridDim.x < B) load(b + gridDim.x);
    if (act_t) {
      for (int q = qh; q < NQ; q += 2) {
        const int py = q / PW, px = q - py * PW;
        const float v = gs[q * C1F_N + n];
        const int m = as[q * C1F_N + n];
        // output pixel (2py + m/2, 2px + m%2); tap (kh, kw) reads x at output + (kh, kw) - pad, i.e.
        // xs[(oy + kh) * LP + ox + kw] in the padded plane
        const float* row = xs + (2 * py + (m >> 1) + kh) * C1F_LP + 2 * px + (m & 1);
#pragma unroll
        for (int kw = 0; kw < KS; ++kw) acc[kw] = __builtin_fmaf(v, row[kw], acc[kw]);
        dbacc += v;
      }
    }
    __syncthreads();
  }
  // the two q parities -> one partial (parity 0 + parity 1, fixed order), db from the kh == 0 threads
  if (qh == 1 && act_t) {
#pragma unroll
    for (int kw = 0; kw < KS; ++kw) red[(kh * C1F_N + n) * KS + kw] = acc[kw];
    if (kh == 0) red[KS * C1F_N * KS + n] = dbacc;
  }
  __syncthreads();
  if (qh == 0 && act_t) {
    float* o = ws + (long)blockIdx.x * LEN;
#pragma unroll
    for (int kw = 0; kw < KS; ++kw) o[n * T + kh * KS + kw] = acc[kw] + red[(kh * C1F_N + n) * KS + kw];
    if (kh == 0) o[C1F_N * T + n] = dbacc + red[KS * C1F_N * KS + n];
  }
}

bool conv1_f32_shape_ok(const ConvGeom& g) {
  return g.C == 1 && g.Cout == C1F_N && (g.KH == 5 || g.KH == 3) && g.KW == g.KH && g.stride == 1 &&
         g.pad == g.KH / 2 && g.OH == g.H && g.OW == g.W && ((g.H | g.W) & 1) == 0 && g.W + g.KW - 1 <= C1F_LP &&
         g.H + g.KH - 1 <= C1F_LP && g.H * g.W <= 1024;
}

}  // namespace

long conv1_wgrad_pooled_f32_ws_floats(int B) {
  return (long)(B < 512 ? B : 512) * (C1F_N * 25 + C1F_N);
}

bool launch_conv1_wgrad_pooled_f32(const float* dp, const uint8_t* am, const float* x, float* dw, float* db, float* ws,
                                   long ws_floats, const ConvGeom& g, float scale, hipStream_t s) {
  if (!conv1_f32_shape_ok(g) || g.B < 1) return false;
  // >= 2 images per workgroup (the next image's loads overlap the current one), at most 2 per CU
  const int grid = std::min(512, (g.B + 1) / 2);
  const int T = g.KH * g.KW, LEN = C1F_N * T + C1F_N;
  if ((long)grid * LEN > ws_floats) return false;
  if (g.KH == 5)
    hipLaunchKernelGGL(conv1_wgrad_pooled_f32_kernel<5>, dim3(grid), dim3(320), 0, s, dp, am, x, ws, g.B, g.H, g.W);
  else
    hipLaunchKernelGGL(conv1_wgrad_pooled_f32_kernel<3>, dim3(grid), dim3(320), 0, s, dp, am, x, ws, g.B, g.H, g.W);
  launch_partials_reduce(ws, grid, LEN, C1F_N * T, dw, db, scale, s);
  return true;
}

void launch_conv_fwd_f32(const ConvF32Args& a, hipStream_t s) {
  const ConvGeom& g = a.g;
  if (g.pool_order && conv1_f32_shape_ok(g)) {  // the 1-channel input layer: conv1_fwd_pool_f32_kernel
    const int grid = std::min(g.B, 1024);
    if (g.KH == 5) hipLaunchKernelGGL(conv1_fwd_pool_f32_kernel<5>, dim3(grid), dim3(256), 0, s, a);
    else hipLaunchKernelGGL(conv1_fwd_pool_f32_kernel<3>, dim3(grid), dim3(256), 0, s, a);
    return;
  }
  const int M = g.B * g.OH * g.OW;
  if (g.Cout <= 32) {
    using Cfg = TileCfg<float, 64, 32, 4, 1>;
    hipLaunchKernelGGL(conv_fwd_f32_kernel<Cfg>, dim3(ntiles<Cfg>(M, g.Cout)), dim3(GEMM_THREADS), 0, s, a);
  } else {
    using Cfg = TileCfg<float, 64, 64, 2, 2>;
    hipLaunchKernelGGL(conv_fwd_f32_kernel<Cfg>, dim3(ntiles<Cfg>(M, g.Cout)), dim3(GEMM_THREADS), 0, s, a);
  }
}

void launch_conv_dgrad_f32(const ConvF32Args& a, hipStream_t s) {
  const ConvGeom& g = a.g;
  const int M = g.B * g.H * g.W;
  if (g.C <= 32) {
    using Cfg = TileCfg<float, 64, 32, 4, 1>;
    hipLaunchKernelGGL(conv_dgrad_f32_kernel<Cfg>, dim3(ntiles<Cfg>(M, g.C)), dim3(GEMM_THREADS), 0, s, a);
  } else {
    using Cfg = TileCfg<float, 64, 64, 2, 2>;
    hipLaunchKernelGGL(conv_dgrad_f32_kernel<Cfg>, dim3(ntiles<Cfg>(M, g.C)), dim3(GEMM_THREADS), 0, s, a);
  }
}

void launch_conv_wgrad_f32(const ConvF32Args& a0, hipStream_t s) {
  ConvF32Args a = a0;
  const ConvGeom& g = a.g;
  using Cfg = TileCfg<float, 32, 64, 2, 2>;
  const int M = g.Cout, N = g.KH * g.KW * g.C + (a.db ? 1 : 0), Kred = g.B * g.OH * g.OW;
  const int tiles = ntiles<Cfg>(M, N);
  // split the pixel reduction so ~2048 workgroups (8 per CU, 2 waves per SIMD each) hide the
  // gather latency, at least 16 k-tiles each (512 workgroups left conv2's weight gradient at 2 per
  // CU and ~30 TFLOP/s, latency-bound)
  int splits = (2048 + tiles - 1) / tiles;
  int chunk = (Kred + splits - 1) / splits;
  chunk = (chunk + BK - 1) / BK * BK;
  if (chunk < 16 * BK) chunk = 16 * BK;
  splits = (Kred + chunk - 1) / chunk;
  a.k_chunk = chunk;
  hipLaunchKernelGGL(conv_wgrad_f32_kernel<Cfg>, dim3(tiles, 1, splits), dim3(GEMM_THREADS), 0, s, a);
}

void launch_unpool_f32(const float* g, const uint8_t* am, float* out, int B, int PH, int PW, int C, hipStream_t s) {
  const long n = (long)B * PH * PW * C;
  hipLaunchKernelGGL(unpool_f32_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, g, am, out, PH, PW, C, n);
}

void launch_transpose_taps_f32(const float* in, float* out, int O, int T, int C, hipStream_t s) {
  const long n = (long)O * T * C;
  hipLaunchKernelGGL(transpose_taps_f32_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, in, out, O, T, C);
}

}  // namespace dtfe
