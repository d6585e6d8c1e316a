// MNIST conv1 (28x28x1 -> 5x5 SAME -> 32 channels) forward (+bias, ReLU, 2x2 max-pool,
// argmax) and weight gradient (dY un-pooled on load), persistent over the batch.
//
// Why a dedicated pair: with one input channel the MFMA reduction index is the tap, so an
// operand fragment (8 consecutive k of one pixel) is 8 horizontally adjacent pixels that start
// at an arbitrary column - the generic few-channel kernels gathered them with 8 ds_read_u16
// and packed them in VALU (rocprof PMC: ~80 VALU per MFMA).  Here each image is staged once
// as a zero-padded plane P and then as S column-shifted copies
//
//     copy_s[r][c] = P[r][c + s + 2]          P[r][c] = X[r - 2][c - 4]
//
// so that "8 pixels from column x" is one aligned ds_read_b128 of copy_(x mod 8) at column
// x - x mod 8 (forward, S = 8) or of copy_kw at column 8g (weight gradient: tap column kw,
// S = 5).  Forward: k = kh*8 + kw (kw >= 5 carry zero weights), two 32-deep MFMA steps per
// 16-pixel tile.  Weight gradient: k = output pixel (one output row of 32 enumerated
// columns per step), A = dY^T through the transposing ds_read_b64_tr_b16, B = shifted copies.
// Both loop over several images per workgroup with the next image's global loads in flight;
// the weight gradient accumulates in registers and flushes one partial per workgroup.
#include "imgconv.h"

#include <stdexcept>
#include <type_traits>

namespace dtfe {

namespace {

constexpr int TH = 256;                  // 4 waves
constexpr int HI = 28;                   // image / output size
constexpr int PWD = 48, PRW = 32;        // P: 32 rows x 48 columns (rows 16-B aligned)
constexpr int CWD = 40;                  // copy row pitch (elements): 5 x 16-B slots
constexpr int CSZ = PRW * CWD + 8;       // copy stride (+1 slot skew per copy)
constexpr int NCH = 32;                  // output channels
constexpr int XCH = HI * HI / 4;         // 8-byte chunks of an image (196)

__device__ __forceinline__ u32x4_t ld16l(const bf16* p) { return *reinterpret_cast<const u32x4_t*>(p); }

// compile-time loop: f(std::integral_constant<int, I>{}) for I in [B, E)
template <int B, int E, typename F>
__device__ __forceinline__ void static_for_c1(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for_c1<B + 1, E>(f);
  }
}

// image b -> P interior (8-byte chunks: 4 pixels of one row; rows are 56 B)
__device__ __forceinline__ void load_img(const bf16* x, long b, u32x2_t& v) {
  if (threadIdx.x < XCH) v = *reinterpret_cast<const u32x2_t*>(x + b * (HI * HI) + threadIdx.x * 4);
}
__device__ __forceinline__ void write_img(bf16* P, const u32x2_t& v) {
  if (threadIdx.x < XCH) {
    const int r = threadIdx.x / 7, c = (threadIdx.x - r * 7) * 4;
    *reinterpret_cast<u32x2_t*>(P + (r + 2) * PWD + c + 4) = v;
  }
}

// copies s < S (rows 0..31, 32 columns each = 4 chunks of 8).  Thread (r, c8, half) reads the three
// aligned 16-B chunks P[r][c8 .. c8+23] once and forms its copies' 8-element windows (first element
// s + 2) with dword funnel shifts (v_alignbyte) - an earlier form gathered every element with its own
// ds_read_u16 (8 LDS reads + 8 VALU per chunk, bank conflicts: rocprof PMC r6pmc2)
__device__ __forceinline__ uint32_t shr16(uint32_t lo, uint32_t hi) {
  return (uint32_t)((((uint64_t)hi << 32) | lo) >> 16);
}
template <int S>
__device__ __forceinline__ void build_copies(const bf16* P, bf16* C) {
  constexpr int HALF = (S + 1) / 2;  // copies per thread: threads 0..127 take s < HALF, 128..255 the rest
  const int t = threadIdx.x & 127, r = t >> 2, c8 = (t & 3) * 8;
  const u32x4_t* src = reinterpret_cast<const u32x4_t*>(P + r * PWD + c8);
  uint32_t d[12];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const u32x4_t v = src[j];
#pragma unroll
    for (int e = 0; e < 4; ++e) d[4 * j + e] = v[e];
  }
  auto emit = [&](auto sc) {
    constexpr int s = decltype(sc)::value;
    constexpr int e0 = s + 2;
    u32x4_t o;
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = (e0 & 1) ? shr16(d[(e0 >> 1) + j], d[(e0 >> 1) + j + 1]) : d[(e0 >> 1) + j];
    *reinterpret_cast<u32x4_t*>(C + s * CSZ + r * CWD + c8) = o;
  };
  if (threadIdx.x < 128) {
    static_for_c1<0, HALF>(emit);
  } else {
    static_for_c1<HALF, S>(emit);
  }
}

// ------------------------------------------------------------------ forward
template <int ACT>  // the epilogue activation is a compile-time constant (a runtime switch per value
                    // was ~a fifth of the kernel's VALU)
__global__ __launch_bounds__(TH) void conv1c_fwd_kernel(ImgConvArgs a) {
  __shared__ __attribute__((aligned(16))) bf16 P[PRW * PWD];
  __shared__ __attribute__((aligned(16))) bf16 C[8 * CSZ];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, g = lane >> 4;
  for (int i = threadIdx.x; i < PRW * PWD / 8; i += TH) reinterpret_cast<u32x4_t*>(P)[i] = u32x4_t{0u, 0u, 0u, 0u};

  // weights as B fragments: step 0 rows kh = g (kw 0..7), step 1 row kh = 4 (g == 0 only)
  bf16x8_t bw[2][2];
  float biasv[2];
#pragma unroll
  for (int nt = 0; nt < 2; ++nt) {
    const int n = nt * 16 + (lane & 15);
    biasv[nt] = a.bias ? a.bias[n] : 0.f;
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      const int kh = st == 0 ? g : 4;
      const bool rowok = st == 0 || g == 0;
      s16x8_t v;
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (short)((rowok && j < 5) ? a.w[n * 25 + kh * 5 + j] : 0);
      bw[nt][st] = __builtin_bit_cast(bf16x8_t, v);
    }
  }

  // fused batch sampling (a.g_src): the sampled uint8 row is converted here and the bf16
  // image written out for the weight gradient - no separate gather launch per step
  const int64_t gstep = a.g_src ? *a.g_counter : 0;
  for (int z = 0; z < ((a.diag & 8) ? 0 : a.nz); ++z)
    for (long i = (long)blockIdx.x * TH + threadIdx.x; i < a.zlen[z]; i += (long)gridDim.x * TH) a.zptr[z][i] = 0u;
  auto load = [&](long bb, u32x2_t& v) {
    if (!a.g_src) {
      load_img(a.src, bb, v);
      return;
    }
    const long r = (long)(hash_u32(a.g_seed, (uint64_t)gstep * a.B + bb) % (uint32_t)a.g_rows);
    if (threadIdx.x < XCH) {
      const uint32_t px = *reinterpret_cast<const uint32_t*>(a.g_src + r * (HI * HI) + threadIdx.x * 4);
      const float k = 1.f / 255.f;
      v = u32x2_t{pack_bf16x2((float)(px & 0xffu) * k, (float)((px >> 8) & 0xffu) * k),
                  pack_bf16x2((float)((px >> 16) & 0xffu) * k, (float)(px >> 24) * k)};
      *reinterpret_cast<u32x2_t*>(const_cast<bf16*>(a.src) + bb * (HI * HI) + threadIdx.x * 4) = v;
    }
    if (threadIdx.x == 0 && a.g_labels_dst) a.g_labels_dst[bb] = a.g_labels_src[r];
  };
  u32x2_t xv = {0u, 0u};
  long b = blockIdx.x;
  if (b < a.B) load(b, xv);
  __syncthreads();
  for (; b < a.B; b += gridDim.x) {
    write_img(P, xv);
    __syncthreads();
    if (b + gridDim.x < a.B) load(b + gridDim.x, xv);
    if (!(a.diag & 2)) build_copies<8>(P, C);
    __syncthreads();
    // 49 tiles of 16 output pixels in 2x2-window order (4 windows per tile)
    for (int t = wid; t < ((a.diag & 4) ? 0 : 49); t += 4) {
      const int m = t * 16 + (lane & 15), q = m & 3, w = m >> 2;
      const int oy = 2 * (w / 14) + (q >> 1), ox = 2 * (w % 14) + (q & 1);
      const int s = ox & 7;
      const bf16* ab = C + s * CSZ + (ox - s) + oy * CWD;
      const bf16x8_t a0 = __builtin_bit_cast(bf16x8_t, ld16l(ab + g * CWD));
      const bf16x8_t a1 = __builtin_bit_cast(bf16x8_t, ld16l(ab + 4 * CWD));
      f32x4_t acc[2];
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, bw[nt][0], f32x4_t{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
        acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, bw[nt][1], acc[nt], 0, 0, 0);
      }
      // lane holds rows (lane>>4)*4 + j = one 2x2 window, column lane & 15 of each n-tile.
      // Direct scattered stores: at 4-6 workgroups per CU they hide behind the other
      // workgroups' MFMAs (an LDS-staged 16-B store epilogue measured 15 -> 19 us here)
      const int wq = t * 4 + g, py = wq / 14, px = wq - py * 14;
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        const f32x4_t v = acc[nt];
        int am = 0;
        float mx = v[0];
#pragma unroll
        for (int j = 1; j < 4; ++j) if (v[j] > mx) { mx = v[j]; am = j; }
        const long o = ((b * 14 + py) * 14 + px) * NCH + nt * 16 + (lane & 15);
        if (a.diag & 1) continue;
        a.y[o] = f2bf(apply_act(mx + biasv[nt], ACT));
        if (a.argmax) a.argmax[o] = (uint8_t)am;
      }
    }
    __syncthreads();
  }
  if (a.g_src && a.g_done && threadIdx.x == 0) {  // the last workgroup advances the sampling step
    const uint32_t prev = __hip_atomic_fetch_add(a.g_done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (prev == gridDim.x - 1) {
      __hip_atomic_fetch_add((unsigned long long*)a.g_counter, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(a.g_done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// ------------------------------------------------------------ weight grad
constexpr int DP = NCH;  // dY image pitch (elements per pixel)

__global__ __launch_bounds__(TH) void conv1c_wgrad_kernel(ImgWgradArgs a, int diag) {
  __shared__ __attribute__((aligned(16))) bf16 P[PRW * PWD];
  __shared__ __attribute__((aligned(16))) bf16 C[5 * CSZ];
  __shared__ __attribute__((aligned(16))) bf16 D[HI * 32 * DP];  // dY [oy][ox < 32][n]
  constexpr int RL = 32 * 32 + 32;      // one wave's partial dW[n][tap < 32] + db[n]
  // the cross-wave partials reuse D (dead after the image loop): ~73 KB of LDS, two workgroups per CU
  static_assert(4 * RL * 4 <= HI * 32 * DP * 2, "partials must fit in the dY image");
  float* red = reinterpret_cast<float*>(D);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, g = lane >> 4, i16 = lane & 15;
  const int q4 = i16 >> 2, p4 = i16 & 3;
  for (int i = threadIdx.x; i < PRW * PWD / 8; i += TH) reinterpret_cast<u32x4_t*>(P)[i] = u32x4_t{0u, 0u, 0u, 0u};
  for (int i = threadIdx.x; i < HI * 32 * DP / 8; i += TH) reinterpret_cast<u32x4_t*>(D)[i] = u32x4_t{0u, 0u, 0u, 0u};

  // B fragment addresses: tap ti = tt*16 + i16 -> (kh, kw); taps >= 25 read tap 24 (dropped)
  int boff[2];
#pragma unroll
  for (int tt = 0; tt < 2; ++tt) {
    const int ti = min(tt * 16 + i16, 24), kh = ti / 5, kw = ti - kh * 5;
    boff[tt] = kw * CSZ + kh * CWD + 8 * g;
  }
  // A (dY^T) transposed-read addresses within one output row: pixels 8g + 4h + q4, columns 4*p4
  int aoff[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) aoff[h] = (8 * g + 4 * h + q4) * DP + 4 * p4;

  f32x4_t acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  // bias gradient: the same A fragments against a B of ones (every column = sum over the row's pixels)
  // - one MFMA per n-tile and row instead of 16 VALU per fragment
  f32x4_t dbacc[2] = {f32x4_t{0.f, 0.f, 0.f, 0.f}, f32x4_t{0.f, 0.f, 0.f, 0.f}};
  bf16x8_t ones;
#pragma unroll
  for (int e = 0; e < 8; ++e) ones[e] = (__bf16)1.0f;

  // pooled dY chunks: 14*14 windows x 4 chunks of 8 channels = 784 per image
  constexpr int PCH = 14 * 14 * (NCH / 8);
  constexpr int NPF = (PCH + TH - 1) / TH;  // 4
  u32x4_t pv[NPF];
  u32x2_t pam[NPF];
  u32x2_t xv = {0u, 0u};
  auto load_all = [&](long b) {
    load_img(a.src, b, xv);
#pragma unroll
    for (int j = 0; j < NPF; ++j) {
      const int i = threadIdx.x + j * TH;
      if (i < PCH) {
        const long o = b * (PCH * 8) + (long)i * 8;
        pv[j] = *reinterpret_cast<const u32x4_t*>(a.dy_pooled + o);
        pam[j] = *reinterpret_cast<const u32x2_t*>(a.dy_argmax + o);
      }
    }
  };
  auto write_dy = [&]() {
#pragma unroll
    for (int j = 0; j < NPF; ++j) {
      const int i = threadIdx.x + j * TH;
      if (i >= PCH) continue;
      const int win = i >> 2, c8 = (i & 3) * 8, py = win / 14, px = win - py * 14;
      u32x4_t v[4];
      unpool4(pv[j], pam[j], v);
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) {
        const int oy = 2 * py + (qq >> 1), ox = 2 * px + (qq & 1);
        // the 32-B channel half of pixel ox is swapped when bit 3 of ox is set: a transposed read's
        // 8 pixels (ox, ox+1, .., ox+3, ox+8, .., ox+11) then cover all 64 banks (64-B pixel pitch
        // put ox and ox+8 on the same banks: 2-way conflicts, r6pmc2)
        *reinterpret_cast<u32x4_t*>(D + (oy * 32 + ox) * DP + (c8 ^ (((ox >> 3) & 1) << 4))) = v[qq];
      }
    }
  };

  long b = blockIdx.x;
  if (b < a.B) load_all(b);
  __syncthreads();
  for (; b < a.B; b += gridDim.x) {
    write_img(P, xv);
    if (!(diag & 1)) write_dy();
    __syncthreads();
    if (b + gridDim.x < a.B) load_all(b + gridDim.x);
    if (!(diag & 2)) build_copies<5>(P, C);
    __syncthreads();
    for (int oy = wid; oy < ((diag & 4) ? 0 : HI); oy += 4) {
      bf16x8_t af[2];
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        const bf16* base = D + oy * 32 * DP + ((nt ^ (g & 1)) * 16);  // (pixel bit 3 = g: write_dy's swap)
        const s16x4_t h0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4_t, base + aoff[0]));
        const s16x4_t h1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4_t, base + aoff[1]));
        const s16x8_t v = {h0[0], h0[1], h0[2], h0[3], h1[0], h1[1], h1[2], h1[3]};
        af[nt] = __builtin_bit_cast(bf16x8_t, v);
        dbacc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[nt], ones, dbacc[nt], 0, 0, 0);
      }
#pragma unroll
      for (int tt = 0; tt < 2; ++tt) {
        const bf16x8_t bf = __builtin_bit_cast(bf16x8_t, ld16l(C + boff[tt] + oy * CWD));
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) acc[nt][tt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[nt], bf, acc[nt][tt], 0, 0, 0);
      }
    }
    __syncthreads();
  }
  if (diag & 8) {  // ablation: keep the loads live without the flush
    if (a.ws && acc[0][0][0] == 12345.f) a.ws[blockIdx.x] = dbacc[0][0];
    return;
  }
  // cross-wave reduction in LDS: every wave stores its own partial (no LDS float atomics), the
  // flush sums the 4 in wave order - the weight gradient is bitwise reproducible
  float* mine = red + wid * RL;
#pragma unroll
  for (int nt = 0; nt < 2; ++nt)
#pragma unroll
    for (int tt = 0; tt < 2; ++tt)
#pragma unroll
      for (int j = 0; j < 4; ++j) mine[(nt * 16 + g * 4 + j) * 32 + tt * 16 + i16] = acc[nt][tt][j];
#pragma unroll
  for (int nt = 0; nt < 2; ++nt)  // column 0 of the ones product: rows 4g..4g+3 of n-tile nt
    if (i16 == 0)
#pragma unroll
      for (int j = 0; j < 4; ++j) mine[32 * 32 + nt * 16 + g * 4 + j] = dbacc[nt][j];
  __syncthreads();
  // flush: dW[n][tap] (tap < 25) and db[n]; one partial per workgroup (summed by the reduce
  // kernel) or, without a workspace, scaled atomics
  constexpr int KC = 25, LEN = NCH * KC + NCH;
  float* part = a.ws ? a.ws + (long)blockIdx.x * LEN : nullptr;
  for (int i = threadIdx.x; i < LEN; i += TH) {
    const int r = i < NCH * KC ? (i / KC) * 32 + (i % KC) : 32 * 32 + (i - NCH * KC);
    const float v = ((red[r] + red[RL + r]) + red[2 * RL + r]) + red[3 * RL + r];
    if (part) part[i] = v;
    else if (i < NCH * KC) atomicAdd(a.dw + i, v * a.scale);
    else if (a.db) atomicAdd(a.db + (i - NCH * KC), v * a.scale);
  }
}

bool mnist_conv1_shape(int B, int SH, int SW, int CS, int OH, int OW, int N, int KH, int KW, int stride, int pad) {
  return B >= 256 && SH == HI && SW == HI && CS == 1 && OH == HI && OW == HI && N == NCH && KH == 5 && KW == 5 &&
         stride == 1 && pad == 2;
}

}  // namespace

bool launch_conv1_copies_fwd(const ImgConvArgs& a, hipStream_t s) {
  if (!mnist_conv1_shape(a.B, a.SH, a.SW, a.CS, a.OH, a.OW, a.N, a.KH, a.KW, a.stride, a.pad)) return false;
  if (!a.src || !a.pool || a.flip_taps || a.dil > 1 || a.relu_mask) return false;
  const int grid = a.B < 1024 ? a.B : 1024;
  static const int diag = diag_bits("c1");
  ImgConvArgs ad = a;
  ad.diag = diag;
  switch (a.act) {
    case ACT_RELU: hipLaunchKernelGGL(conv1c_fwd_kernel<ACT_RELU>, dim3(grid), dim3(TH), 0, s, ad); break;
    case ACT_NONE: hipLaunchKernelGGL(conv1c_fwd_kernel<ACT_NONE>, dim3(grid), dim3(TH), 0, s, ad); break;
    default: return false;  // sigmoid / tanh: the generic few-channel kernel
  }
  return true;
}

bool launch_conv1_copies_wgrad(const ImgWgradArgs& a, hipStream_t s) {
  if (!mnist_conv1_shape(a.B, a.SH, a.SW, a.CS, a.OH, a.OW, a.N, a.KH, a.KW, a.stride, a.pad)) return false;
  if (!a.src || a.dy || !a.dy_pooled) return false;
  // DTFE_C1W_GRID: workgroups (images per workgroup = B / grid); DTFE_DIAG c1w=<bits>: ablation bits
  // (1 skip the un-pooled dY image, 2 skip the shifted copies, 4 skip the MFMA tiles, 8 skip the flush)
  static const int want = [] {
    const char* e = getenv("DTFE_C1W_GRID");
    return e ? atoi(e) : 320;  // beside conv2's weight gradient: 320 / 384 ~0.8 % faster than 256 (r3zg)
  }();
  static const int diag = diag_bits("c1w");
  const int grid = a.B < want ? a.B : (want < 1 ? 1 : want);
  if (a.ws && (long)grid * (NCH * 25 + NCH) > imgwgrad_ws_floats(NCH, 25))
    throw std::runtime_error("conv1 wgrad: partials exceed the workspace");
  hipLaunchKernelGGL(conv1c_wgrad_kernel, dim3(grid), dim3(TH), 0, s, a, diag);
  if (a.ws) {
    constexpr int LEN = NCH * 25 + NCH;
    launch_partials_reduce(a.ws, grid, LEN, NCH * 25, a.dw, a.db, a.scale, s);
  }
  return true;
}

}  // namespace dtfe
