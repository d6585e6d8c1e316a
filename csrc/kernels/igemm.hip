// Implicit-GEMM NHWC convolution for wide layers on gfx950 (see igemm.h).
//
// Main loop ("2-buffer glds" structure of the CDNA4 guide, §5): 4 waves, a
// BM x BN output tile, 64-deep k-tiles.  Both operands of a k-tile are moved
// HBM -> LDS by global_load_lds_dwordx4 (16 B per lane, no VGPR staging), tile
// t+1 is in flight while the MFMAs of tile t run, one barrier per k-tile.
//
// LDS images are lane-linear (the DMA writes base + 16*lane), so the bank
// swizzle is applied on the SOURCE address and undone on the fragment read:
//   fwd/dgrad images [rows][64 k] (128-B rows): LDS slot s of row r holds
//     logical 16-B chunk s ^ (r & 7)  -> the 16x16x32 A/B fragment reads
//     (ds_read_b128, rows r..r+15 at one chunk) hit 16 distinct bank slots
//   wgrad images [64 m][cols] read with ds_read_b64_tr_b16: 32-B segments of
//     m-row k are XOR-ed by h(k) = (k & 3) | ((k >> 3) & 1) << 2 (256-B rows) or
//     ((k >> 1) & 1) | ((k >> 3) & 1) << 1 (128-B rows): the 8 m-rows one
//     32-lane half reads land on 8 distinct 32-B bank segments.
// Out-of-image taps (padding) and rows past the end read a zero page.
//
// Replaces Conv2D / Conv2DBackpropInput / Conv2DBackpropFilter of the ResNet-50
// configuration (BASELINE.json config 5).
#include "igemm.h"
#include "bn_chan.h"

#include <algorithm>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <vector>

namespace dtfe {

namespace {

constexpr int IG_THREADS = 256;
constexpr int IG_BK = 64;

typedef __attribute__((address_space(3))) void lds_void_t;

__device__ __forceinline__ void glds16(const void* g, bf16* lds_piece) {
  __builtin_amdgcn_global_load_lds(g, (lds_void_t*)lds_piece, 16, 0, 0);
}

// The same DMA issued from inline asm (M0 = the wave-uniform LDS destination): invisible to the
// compiler's LDS-DMA alias tracking, which otherwise puts an `s_waitcnt vmcnt(0)` in front of the
// first fragment read of every k-tile of a multi-stage ring (it cannot tell the stage being filled
// from the one being read) and so drains the prefetch.  The caller orders every DMA'd tile with
// its own counted vmcnt wait + barrier; the compiler's own waits stay conservative (these DMAs
// are always older than the loads it counts).
__device__ __forceinline__ void glds16_async(const void* g, bf16* lds_piece) {
  const uint32_t l = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)lds_piece);
  asm volatile("global_load_lds_dwordx4 %0, off" ::"v"(g), "{m0}"(l) : "memory");
}

// exact m / d for 0 <= m < 2^24 through a float reciprocal
__device__ __forceinline__ int qdiv(int m, int d, float inv_d) {
  int q = (int)((float)m * inv_d);
  const int r = m - q * d;
  q += (r >= d) - (r < 0);
  return q;
}

// ------------------------------------------------------------ fwd / dgrad
// Epilogue shared by the 4- and 8-wave kernels: fp32 split-K partial tile, or the bf16 tile through
// LDS (+ accumulation source, BatchNorm forward / backward partial statistics).  THREADS threads,
// a 2-column wave grid (wave w owns rows (w >> 1) * WM.., columns (w & 1) * WN..).
template <int BM, int BN, int THREADS, int SMEM_EL, bool BB>
__device__ __forceinline__ void igemm_store(const IgemmArgs& a, const f32x4_t (&acc)[BM / (THREADS / 128) / 16][BN / 2 / 16],
                                            bf16* smem, int tid, int lane, int w, int m_base, int n_base,
                                            int tm, int Mp, const IgPhase& P) {
  constexpr int IG_THREADS = THREADS;
  constexpr int WM = BM / (THREADS / 128), WN = BN / 2, TM = WM / 16, TN = WN / 16;
  const int wm = w >> 1, wn = w & 1;
  if (a.splits > 1) {
    // fp32 partial tile (forward only: one phase, output row == m)
    float* ws = a.ws + (long)blockIdx.y * Mp * a.N;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = n_base + wn * WN + j * 16 + (lane & 15);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int m = m_base + wm * WM + i * 16 + (lane >> 4) * 4 + q;
          if (m < Mp) ws[(long)m * a.N + col] = acc[i][j][q];
        }
      }
    return;
  }

  // output addresses and every epilogue operand load (accumulation source, BN-backward x / y) are
  // issued before the C tile is staged, so their latency hides under the LDS round trip
  constexpr int CPR = BN / 8;
  constexpr int PER = BM * CPR / IG_THREADS;  // 16-B chunks per thread
  static_assert(PER * IG_THREADS == BM * CPR, "whole chunks per thread");
  bf16* dst[PER];
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int q = tid + j * IG_THREADS, r = q / CPR, c8 = q - r * CPR;
    const int m = m_base + r;
    dst[j] = nullptr;
    if (m >= Mp) continue;
    long opix = m;
    if (a.ostr > 1) {  // data gradient of a strided conv: phase pixel grid -> output pixel
      const int jx = m % P.RW, t = m / P.RW;
      const int i = t % P.RH, b = t / P.RH;
      opix = ((long)b * a.OHf + i * a.ostr + P.oy) * a.OWf + jx * a.ostr + P.ox;
    }
    dst[j] = a.out + opix * a.N + n_base + c8 * 8;
  }
  u32x4_t old[PER];
  if (a.accum) {  // e.g. a block's input gradient: the shortcut branch's share is already there;
                  // every load is issued before the first add (no per-chunk latency chain)
    if (a.acc_src) {  // ... or computed here: the masked shortcut gradient at the same position
      uint32_t mk[PER];
#pragma unroll
      for (int j = 0; j < PER; ++j) {
        const long off = dst[j] ? (long)(dst[j] - a.out) : 0;
        old[j] = *reinterpret_cast<const u32x4_t*>(a.acc_src + off);
        mk[j] = a.acc_mask[off >> 3];
      }
#pragma unroll
      for (int j = 0; j < PER; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e)
          old[j][e] &= ((mk[j] >> (2 * e)) & 1u ? 0x0000ffffu : 0u) | ((mk[j] >> (2 * e + 1)) & 1u ? 0xffff0000u : 0u);
    } else {
#pragma unroll
      for (int j = 0; j < PER; ++j) old[j] = dst[j] ? *reinterpret_cast<const u32x4_t*>(dst[j]) : u32x4_t{0u, 0u, 0u, 0u};
    }
  }
  // BatchNorm-backward statistics of the final values: this thread's 8 channels are the same for
  // every j (IG_THREADS % CPR == 0); x (and y for a non-recomputable mask) at the same offsets
  const bool bb = BB && a.bb_x != nullptr;  // compiled out of the instances without a BN-backward epilogue
  const bool bb_from_x = bb && a.bb_y == nullptr && a.bb_act == ACT_RELU;
  const bool bb_need_y = bb && a.bb_act != ACT_NONE && !bb_from_x;
  u32x4_t xv[PER], yv[PER];
  float bmean[8], binv[8], bsc[8], bsh[8], bs[8] = {}, bq[8] = {};
  const int my_c8 = tid % CPR;
  if (bb) {
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const long off = dst[j] ? (long)(dst[j] - a.out) : 0;
      xv[j] = *reinterpret_cast<const u32x4_t*>(a.bb_x + off);
      if (bb_need_y) yv[j] = *reinterpret_cast<const u32x4_t*>(a.bb_y + off);
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int c = n_base + my_c8 * 8 + e;
      bmean[e] = a.bb_mean[c];
      binv[e] = a.bb_invstd[c];
      if (bb_from_x) {  // = norm.hip BwdMask (bit-identical to the forward's pre-activation)
        bsc[e] = a.bb_gamma[c] * a.bb_invstd[c];
        bsh[e] = bn_shift(a.bb_beta[c], a.bb_mean[c], bsc[e]);
      }
    }
  }
  // bf16 tile through LDS, then 16-B row-contiguous stores
  constexpr int CLD = BN + 8;
  static_assert(BM * CLD <= SMEM_EL, "C tile fits the staging LDS");
  __syncthreads();
  bf16* Cs = smem;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        Cs[(wm * WM + i * 16 + (lane >> 4) * 4 + q) * CLD + wn * WN + j * 16 + (lane & 15)] = f2bf(acc[i][j][q]);
  __syncthreads();
  if (a.bn_part && !a.bb_x) {
    // BatchNorm statistics of this tile's stored values (replaces a separate pass over y):
    // thread = (8-channel chunk, row group); sums around the tile's first row, then the row
    // groups in order through the LDS past the C tile (deterministic)
    constexpr int CH = BN / 8, RG = IG_THREADS / CH;
    static_assert(BM * CLD * 2 + RG * 2 * BN * 4 <= SMEM_EL * 2, "stats scratch fits");
    float* red = reinterpret_cast<float*>(smem + BM * CLD);
    const int ch = tid % CH, rg = tid / CH, rows = min(BM, Mp - m_base);
    float k[8], sm[8] = {}, sq[8] = {};
    const u32x4_t kv = *reinterpret_cast<const u32x4_t*>(Cs + ch * 8);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      k[2 * e] = bf2f((bf16)(kv[e] & 0xffffu));
      k[2 * e + 1] = bf2f((bf16)(kv[e] >> 16));
    }
    for (int r = rg; r < rows; r += RG) {
      const u32x4_t v = *reinterpret_cast<const u32x4_t*>(Cs + r * CLD + ch * 8);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float d0 = bf2f((bf16)(v[e] & 0xffffu)) - k[2 * e], d1 = bf2f((bf16)(v[e] >> 16)) - k[2 * e + 1];
        sm[2 * e] += d0; sq[2 * e] += d0 * d0;
        sm[2 * e + 1] += d1; sq[2 * e + 1] += d1 * d1;
      }
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      red[(rg * 2) * BN + ch * 8 + e] = sm[e];
      red[(rg * 2 + 1) * BN + ch * 8 + e] = sq[e];
    }
    __syncthreads();
    for (int c = tid; c < BN; c += IG_THREADS) {
      float S = 0.f, Q = 0.f;
      for (int g2 = 0; g2 < RG; ++g2) {
        S += red[(g2 * 2) * BN + c];
        Q += red[(g2 * 2 + 1) * BN + c];
      }
      float* pp = a.bn_part + (long)tm * 3 * a.N + n_base + c;
      pp[0] = bf2f(Cs[c]);
      pp[a.N] = S;
      pp[2 * a.N] = Q;
    }
  }
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    if (!dst[j]) continue;
    const int q = tid + j * IG_THREADS, r = q / CPR, c8 = q - r * CPR;
    u32x4_t v = *reinterpret_cast<const u32x4_t*>(Cs + r * CLD + c8 * 8);
    if (a.accum) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float lo = bf2f((bf16)(v[e] & 0xffffu)) + bf2f((bf16)(old[j][e] & 0xffffu));
        const float hi = bf2f((bf16)(v[e] >> 16)) + bf2f((bf16)(old[j][e] >> 16));
        v[e] = pack_bf16x2(lo, hi);
      }
    }
    *reinterpret_cast<u32x4_t*>(dst[j]) = v;
    if (bb) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float g0 = bf2f((bf16)((v[e >> 1] >> (16 * (e & 1))) & 0xffffu));
        const float x = bf2f((bf16)((xv[j][e >> 1] >> (16 * (e & 1))) & 0xffffu));
        float g = g0;
        if (bb_from_x) {
          g = bn_affine(x, bsc[e], bsh[e]) > 0.f ? g0 : 0.f;
        } else if (a.bb_act != ACT_NONE) {
          g = g0 * act_grad_from_out(bf2f((bf16)((yv[j][e >> 1] >> (16 * (e & 1))) & 0xffffu)), a.bb_act);
        }
        bs[e] += g;
        bq[e] += g * (x - bmean[e]) * binv[e];
      }
    }
  }
  if (bb) {  // row groups -> per-tile partial, fixed order, through the LDS past the C tile
    constexpr int RG = IG_THREADS / CPR;
    static_assert(BM * CLD * 2 + RG * 2 * BN * 4 <= SMEM_EL * 2, "bwd stats scratch fits");
    float* red = reinterpret_cast<float*>(smem + BM * CLD);
    const int rg = tid / CPR;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      red[(rg * 2) * BN + my_c8 * 8 + e] = bs[e];
      red[(rg * 2 + 1) * BN + my_c8 * 8 + e] = bq[e];
    }
    __syncthreads();
    float* pp = a.bn_part + ((long)blockIdx.z * a.tiles_m + tm) * 3 * a.N + n_base;
    for (int c = tid; c < BN; c += IG_THREADS) {
      float S = 0.f, Q = 0.f;
      for (int g2 = 0; g2 < RG; ++g2) {
        S += red[(g2 * 2) * BN + c];
        Q += red[(g2 * 2 + 1) * BN + c];
      }
      pp[c] = 0.f;
      pp[a.N + c] = S;
      pp[2 * a.N + c] = Q;
    }
  }
}

// NST: LDS stages (1 only for launches whose every workgroup has ONE k-tile: the 64-channel 1x1
// convs - half the LDS, so three workgroups share a CU instead of two); BB: with the BN-backward
// statistics epilogue (its registers are compiled out of the other instances); MINB: workgroups
// per CU the register allocation must allow
template <int BM, int BN, int NST, bool BB>
constexpr int ig_smem_el() {
  constexpr int stage = NST * (BM + BN) * IG_BK, cld = BN + 8, rg = IG_THREADS / (BN / 8);
  constexpr int epi = (BM * cld * 2 + rg * 2 * BN * 4 + 3) / 4 * 2;  // C tile + statistics scratch, in bf16 units
  return stage > epi ? stage : epi;
}

template <int BM, int BN, int NST, bool BB, int MINB>
__global__ __launch_bounds__(IG_THREADS, MINB) void igemm_kernel(const IgemmArgs a) {
  constexpr int WM = BM / 2, WN = BN / 2, TM = WM / 16, TN = WN / 16;
  constexpr int A_EL = BM * IG_BK, B_EL = BN * IG_BK;
  constexpr int NA = BM / 32, NB = BN / 32;  // 1-KB glds pieces per thread and k-tile
  constexpr int SMEM_EL = ig_smem_el<BM, BN, NST, BB>();
  __shared__ __attribute__((aligned(16))) bf16 smem[SMEM_EL];

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tiles_n = a.N / BN;
  const int id = xcd_remap(blockIdx.x, a.tiles_m * tiles_n);
  const int tm = id / tiles_n, tn = id - tm * tiles_n;
  const IgPhase& P = a.ph[blockIdx.z];
  const int Mp = a.B * P.RH * P.RW;
  const int m_base = tm * BM, n_base = tn * BN;
  if (m_base >= Mp) {
    if (a.bb_x) {  // a phase with fewer tiles: its absent tiles contribute zero BN-backward partials
      float* pp = a.bn_part + ((long)blockIdx.z * a.tiles_m + tm) * 3 * a.N + n_base;
      for (int c = tid; c < BN; c += IG_THREADS) pp[c] = pp[a.N + c] = pp[2 * a.N + c] = 0.f;
    }
    return;
  }

  const int cpt = a.SC / IG_BK;
  const int nk_all = P.ntaps * cpt;
  const int kt0 = (int)((long)nk_all * blockIdx.y / a.splits);
  const int nk = (int)((long)nk_all * (blockIdx.y + 1) / a.splits) - kt0;

  // lane -> (row of an 8-row piece, logical 16-B chunk it fetches)
  const int lrow = lane >> 3, lchunk = (lane & 7) ^ lrow;
  int a_pix[NA], a_iy[NA], a_ix[NA];
#pragma unroll
  for (int j = 0; j < NA; ++j) {
    const int m = m_base + (j * 4 + w) * 8 + lrow;
    a_pix[j] = 0;
    a_iy[j] = -(1 << 20);
    a_ix[j] = 0;
    if (m < Mp) {
      const int jx = m % P.RW, t = m / P.RW;
      const int i = t % P.RH, b = t / P.RH;
      a_pix[j] = b * a.SH * a.SW;
      a_iy[j] = i * a.istr;
      a_ix[j] = jx * a.istr;
    }
  }
  const bf16* b_src[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) b_src[j] = a.w + (long)(n_base + (j * 4 + w) * 8 + lrow) * a.Ktot + lchunk * 8;

  auto issue = [&](int kt, int buf) {
    const int tap = kt / cpt, cb = kt - tap * cpt;
    const int dy = P.dy[tap], dx = P.dx[tap];
    const int woff = P.kt[tap] * a.SC + cb * IG_BK;
    bf16* As = smem + buf * (A_EL + B_EL);
    bf16* Bs = As + A_EL;
#pragma unroll
    for (int j = 0; j < NA; ++j) {
      const int sy = a_iy[j] + dy, sx = a_ix[j] + dx;
      const bool ok = (unsigned)sy < (unsigned)a.SH && (unsigned)sx < (unsigned)a.SW;
      const bf16* p = ok ? a.src + (long)(a_pix[j] + sy * a.SW + sx) * a.SC + cb * IG_BK + lchunk * 8 : a.zeros;
      glds16(p, As + (j * 4 + w) * 512);
    }
#pragma unroll
    for (int j = 0; j < NB; ++j) glds16(b_src[j] + woff, Bs + (j * 4 + w) * 512);
  };
  const int wm = w >> 1, wn = w & 1;
  f32x4_t acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  if (nk > 0) issue(kt0, 0);
  for (int t = 0; t < nk; ++t) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (NST > 1 && t + 1 < nk) issue(kt0 + t + 1, (t + 1) & 1);
    const bf16* As = smem + (NST > 1 ? (t & 1) : 0) * (A_EL + B_EL);
    const bf16* Bs = As + A_EL;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int pc = (kk * 4 + (lane >> 4)) ^ (lane & 7);
      bf16x8_t af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i)
        af[i] = *reinterpret_cast<const bf16x8_t*>(As + (wm * WM + i * 16 + (lane & 15)) * IG_BK + pc * 8);
#pragma unroll
      for (int j = 0; j < TN; ++j)
        bfr[j] = *reinterpret_cast<const bf16x8_t*>(Bs + (wn * WN + j * 16 + (lane & 15)) * IG_BK + pc * 8);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  }

  igemm_store<BM, BN, IG_THREADS, SMEM_EL, BB>(a, acc, smem, tid, lane, w, m_base, n_base, tm, Mp, P);
}

// out[i] = bf16(sum_s ws[s][i])   (accum: out[i] = bf16(out[i] + sum_s ws[s][i]))
__global__ __launch_bounds__(256) void splitk_to_bf16_kernel(const float* __restrict__ ws, int splits, long len,
                                                             bf16* __restrict__ out, int accum) {
  const long i = ((long)blockIdx.x * 256 + threadIdx.x) * 4;
  if (i >= len) return;
  f32x4_t v = *reinterpret_cast<const f32x4_t*>(ws + i);
  for (int s = 1; s < splits; ++s) v += *reinterpret_cast<const f32x4_t*>(ws + (long)s * len + i);
  if (accum) {
    const u32x2_t o = *reinterpret_cast<const u32x2_t*>(out + i);
    v[0] += bf2f((bf16)(o[0] & 0xffffu)); v[1] += bf2f((bf16)(o[0] >> 16));
    v[2] += bf2f((bf16)(o[1] & 0xffffu)); v[3] += bf2f((bf16)(o[1] >> 16));
  }
  u32x2_t o = {pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3])};
  *reinterpret_cast<u32x2_t*>(out + i) = o;
}

// ------------------------------------------------------------------ wgrad
// swizzle (16-B chunk XOR) of m-row k in a [64][COLS] image
template <int COLS> __device__ __forceinline__ int wg_swz(int k) {
  if constexpr (COLS == 128) return 2 * ((k & 3) | (((k >> 3) & 1) << 2));
  else return 2 * (((k >> 1) & 1) | (((k >> 3) & 1) << 1));
}

// fragment of a [64 m][COLS] image for rows (output dims) rbase.., k = m rows kk..kk+31
template <int COLS>
__device__ __forceinline__ bf16x8_t wg_frag(const bf16* img, int rbase, int kk, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int c = rbase + 4 * p;
  const int k0 = kk + 8 * g + q, k1 = k0 + 4;
  const bf16* p0 = img + k0 * COLS + (c ^ (wg_swz<COLS>(k0) * 8));
  const bf16* p1 = img + k1 * COLS + (c ^ (wg_swz<COLS>(k1) * 8));
  s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4_t, p0));
  s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4_t, p1));
  s16x8_t v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8_t, v);
}

// BM output channels x BN input channels of one tap; k-tiles of BKW pixels (m rows), an NS-stage LDS
// ring: NS-1 k-tiles in flight behind counted vmcnt waits and a raw barrier (the 2-stage
// vmcnt(0)-per-k-tile loop spent 50-72 % of its wave cycles waiting: profiles/r3_pmc_resnet50_igemm.csv)
template <int N>
__device__ __forceinline__ void wg_wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int BM, int BN, int BKW, int NS, int MINB>
__global__ __launch_bounds__(IG_THREADS, MINB) void igemm_wgrad_kernel(const IgWgradArgs a, float* dw, float scale) {
  constexpr int WM = BM / 2, WN = BN / 2, TM = WM / 16, TN = WN / 16;
  constexpr int A_EL = BKW * BM, B_EL = BKW * BN, ST_EL = A_EL + B_EL;
  constexpr int CPA = BM / 8, RPA = 64 / CPA, NA = BKW * BM / 2048;  // chunks per m-row, m-rows per piece
  constexpr int CPB = BN / 8, RPB = 64 / CPB, NB = BKW * BN / 2048;
  constexpr int P = NA + NB;
  static_assert(NA >= 1 && NB >= 1, "one DMA piece per wave at least");
  __shared__ __attribute__((aligned(16))) bf16 smem[NS * ST_EL];

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int cblocks = a.C / BN;
  const int tiles_n = a.KH * a.KW * cblocks;
  const int id = xcd_remap(blockIdx.x, (a.Cout / BM) * tiles_n);
  const int tm = id / tiles_n, tn = id - tm * tiles_n;
  const int tap = tn / cblocks, cb = tn - tap * cblocks;
  const int kh = tap / a.KW, kw = tap - kh * a.KW;
  const int M = a.B * a.OH * a.OW;
  const int m0 = blockIdx.y * a.mchunk, m1 = min(M, m0 + a.mchunk);
  const int nk = (m1 - m0 + BKW - 1) / BKW;
  const float inv_ow = 1.f / (float)a.OW, inv_oh = 1.f / (float)a.OH;

  // this lane's m-row within each piece and the logical chunk it fetches
  int a_row[NA], a_chk[NA], b_row[NB], b_chk[NB];
#pragma unroll
  for (int j = 0; j < NA; ++j) {
    a_row[j] = (j * 4 + w) * RPA + lane / CPA;
    a_chk[j] = (lane % CPA) ^ wg_swz<BM>(a_row[j]);
  }
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    b_row[j] = (j * 4 + w) * RPB + lane / CPB;
    b_chk[j] = (lane % CPB) ^ wg_swz<BN>(b_row[j]);
  }
  const bf16* dy_col = a.dy + tm * BM;
  const bf16* x_col = a.x + cb * BN;
  auto issue = [&](int t) {
    bf16* As = smem + (t % NS) * ST_EL;
    bf16* Bs = As + A_EL;
    const int mt = m0 + t * BKW;
#pragma unroll
    for (int j = 0; j < NA; ++j) {
      const int m = mt + a_row[j];
      const bf16* p = m < m1 ? dy_col + (long)m * a.Cout + a_chk[j] * 8 : a.zeros;
      glds16_async(p, As + (j * 4 + w) * 512);
    }
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int m = mt + b_row[j];
      const bf16* p = a.zeros;
      if (m < m1) {
        const int q1 = qdiv(m, a.OW, inv_ow);
        const int ox = m - q1 * a.OW;
        const int b = qdiv(q1, a.OH, inv_oh);
        const int oy = q1 - b * a.OH;
        const int sy = oy * a.stride - a.pad + kh, sx = ox * a.stride - a.pad + kw;
        if ((unsigned)sy < (unsigned)a.H && (unsigned)sx < (unsigned)a.W)
          p = x_col + ((long)(b * a.H + sy) * a.W + sx) * a.C + b_chk[j] * 8;
      }
      glds16_async(p, Bs + (j * 4 + w) * 512);
    }
  };

  const int wm = w >> 1, wn = w & 1;
  f32x4_t acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int t = 0; t < NS - 1; ++t)
    if (t < nk) issue(t);
  for (int t = 0; t < nk; ++t) {
    if (t + NS - 2 < nk) wg_wait_vm<(NS - 2) * P>();
    else wg_wait_vm<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // k-tile t landed for every wave; stage (t-1) % NS read by every wave
    __builtin_amdgcn_sched_barrier(0);
    if (t + NS - 1 < nk) issue(t + NS - 1);
    const bf16* As = smem + (t % NS) * ST_EL;
    const bf16* Bs = As + A_EL;
#pragma unroll
    for (int kk = 0; kk < BKW; kk += 32) {
      bf16x8_t af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = wg_frag<BM>(As, wm * WM + i * 16, kk, lane);
#pragma unroll
      for (int j = 0; j < TN; ++j) bfr[j] = wg_frag<BN>(Bs, wn * WN + j * 16, kk, lane);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  }

  const int Kw = a.KH * a.KW * a.C;
  const int col_base = tap * a.C + cb * BN + wn * WN;
  const int row_base = tm * BM + wm * WM;
  if (a.splits == 1) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          float* d = dw + (long)(row_base + i * 16 + (lane >> 4) * 4 + q) * Kw + col_base + j * 16 + (lane & 15);
          *d += scale * acc[i][j][q];
        }
    return;
  }
  float* ws = a.ws + (long)blockIdx.y * a.Cout * Kw;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        ws[(long)(row_base + i * 16 + (lane >> 4) * 4 + q) * Kw + col_base + j * 16 + (lane & 15)] = acc[i][j][q];
}

// ------------------------------------------------------- 3x3 / stride-1 weight gradient, all taps
// dW[co][tap][c] for a 64-channel (co) x 64-channel (c) tile and ALL 9 taps in one workgroup: a
// k-tile is R = 64 / W whole output rows (R*W <= 64 pixels, the rest zero), the dY rows are staged
// once ([64 k][64 co]) and the source rows they need ONCE as a halo'd patch [(R+2) x (W+2) pixels]
// [64 c]; the 9 taps' B fragments are the same patch read at 9 pixel shifts.  Against the per-tap
// kernel (9 workgroups each staging their own shifted source tile and re-staging dY, 2 fragment
// reads per MFMA) this stages 2.6x fewer bytes and reads 0.72 fragments per MFMA.
// Wave w owns c = 16w..16w+15 of the tile for every co (4 tiles) and tap: 36 accumulators.
constexpr int W3_PATCH = 192;  // patch pixels staged per k-tile (>= (R+2)(W+2) for every W <= 64)

// chunk XOR of patch pixel `pix` ([pixel][64 c] image, 128-B rows): the 8 pixels one 32-lane half of
// a transposing read covers (pix..pix+3, pix+8..pix+11 between row wraps) land on distinct
// (bank-row half, 32-B segment) pairs - the 64-column form of wg_swz
__device__ __forceinline__ int w3_swz(int pix) { return wg_swz<64>(pix); }

__global__ __launch_bounds__(IG_THREADS, 1) void igemm_wgrad3_kernel(const IgWgradArgs a, float* dw, float scale,
                                                                    int R, int ktiles_per_img) {
  constexpr int A_EL = 64 * 64, P_EL = W3_PATCH * 64, ST_EL = A_EL + P_EL;
  __shared__ __attribute__((aligned(16))) bf16 smem[2 * ST_EL];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int H = a.H, W = a.W, PW = W + 2;
  const int npix = (R + 2) * PW, kvalid = R * W;
  const int cblocks = a.C / 64;
  const int id = xcd_remap(blockIdx.x, (a.Cout / 64) * cblocks);
  const int tco = id / cblocks, tc = id - tco * cblocks;
  const int T = a.B * ktiles_per_img;
  const int t0 = (int)((long)T * blockIdx.y / a.splits), nk = (int)((long)T * (blockIdx.y + 1) / a.splits) - t0;

  // A rows (2 pieces per thread): k = row -> (r, x) of the k-tile
  int a_r[2], a_x[2], a_chk[2];
  bool a_ok[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int row = (j * 4 + w) * 8 + (lane >> 3);
    a_ok[j] = row < kvalid;
    a_r[j] = a_ok[j] ? row / W : 0;
    a_x[j] = a_ok[j] ? row - a_r[j] * W : 0;
    a_chk[j] = (lane & 7) ^ wg_swz<64>(row);
  }
  // patch pixels (6 pieces per thread): pixel -> (pr, pc) of the halo'd patch
  int p_r[6], p_c[6], p_chk[6];
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    const int pix = (j * 4 + w) * 8 + (lane >> 3);
    p_r[j] = pix < npix ? pix / PW : -(1 << 20);
    p_c[j] = pix < npix ? pix - (pix / PW) * PW : 0;
    p_chk[j] = (lane & 7) ^ w3_swz(pix);
  }
  const bf16* dy_col = a.dy + tco * 64;
  const bf16* x_col = a.x + tc * 64;
  auto issue = [&](int t, int buf) {
    const int kt = t0 + t, b = kt / ktiles_per_img, oy0 = (kt - b * ktiles_per_img) * R;
    bf16* As = smem + buf * ST_EL;
    bf16* Ps = As + A_EL;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int oy = oy0 + a_r[j];
      const bf16* p = (a_ok[j] && oy < H) ? dy_col + ((long)(b * H + oy) * W + a_x[j]) * a.Cout + a_chk[j] * 8 : a.zeros;
      glds16_async(p, As + (j * 4 + w) * 512);
    }
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      const int sy = oy0 - 1 + p_r[j], sx = p_c[j] - 1;
      const bf16* p = ((unsigned)sy < (unsigned)H && (unsigned)sx < (unsigned)W)
                          ? x_col + ((long)(b * H + sy) * W + sx) * a.C + p_chk[j] * 8
                          : a.zeros;
      glds16_async(p, Ps + (j * 4 + w) * 512);
    }
  };

  // B fragment read offsets: lane (g, q, p4) of read half h covers k = kk + 8g + 4h + q at columns
  // 16w + 4p4 .. +3; the patch pixel of k for tap (kh, kw) is pix(k) + kh * PW + kw
  const int g = lane >> 4, q = (lane & 15) >> 2, p4 = lane & 3;
  const int ccol = 16 * w + 4 * p4;
  int boff[2][2][9];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int k = kk * 32 + 8 * g + 4 * h + q;
      const int r = k / W, x = k - r * W;
      const int base = (k < kvalid) ? r * PW + x : 0;  // dead rows (dY is 0): any staged, finite pixel
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int pix = base + (tap / 3) * PW + (tap % 3);
        boff[kk][h][tap] = pix * 64 + (ccol ^ (w3_swz(pix) * 8));
      }
    }

  f32x4_t acc[4][9];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 9; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  if (nk > 0) issue(0, 0);
  for (int t = 0; t < nk; ++t) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t + 1 < nk) issue(t + 1, (t + 1) & 1);
    const bf16* As = smem + (t & 1) * ST_EL;
    const bf16* Ps = As + A_EL;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8_t af[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = wg_frag<64>(As, i * 16, kk * 32, lane);
#pragma unroll
      for (int kh = 0; kh < 3; ++kh) {
        bf16x8_t bfr[3];
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) {
          const s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4_t, Ps + boff[kk][0][kh * 3 + kw]));
          const s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4_t, Ps + boff[kk][1][kh * 3 + kw]));
          const s16x8_t v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          bfr[kw] = __builtin_bit_cast(bf16x8_t, v);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int kw = 0; kw < 3; ++kw)
            acc[i][kh * 3 + kw] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[kw], acc[i][kh * 3 + kw], 0, 0, 0);
      }
    }
  }

  // dW[co][tap][c]: rows co = 16i + 4(lane>>4) + e, column tap*C + c
  const int Kw = 9 * a.C;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int tap = 0; tap < 9; ++tap)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const long o = (long)(tco * 64 + i * 16 + (lane >> 4) * 4 + e) * Kw + tap * a.C + tc * 64 + 16 * w + (lane & 15);
        if (a.splits == 1) dw[o] += scale * acc[i][tap][e];
        else a.ws[(long)blockIdx.y * a.Cout * Kw + o] = acc[i][tap][e];
      }
}

// dw[i] += scale * sum_s ws[s][i]
constexpr int WG_RCH = 8;
// dw[i] += scale * sum_s ws[s][i].  A workgroup covers P = 256 / S float4 positions with S split
// slices per position (thread = (slice, position)): a small weight with many m-splits (e.g. 64x64x1x1
// over 100+ splits: a handful of position-only workgroups, each walking every split serially) still
// fills the chip.  Slices sum their splits in order, then slice 0 adds the S slice sums in order
// through LDS - a fixed summation order (bitwise reproducible).
template <int S>
__global__ __launch_bounds__(256) void wgrad_splits_reduce_kernel(const float* __restrict__ ws, int splits, long len,
                                                                  float* dw, float scale) {
  constexpr int P = 256 / S;
  __shared__ f32x4_t red[S > 1 ? S : 1][P];
  const int pos = threadIdx.x % P, sl = threadIdx.x / P;
  const long i = ((long)blockIdx.x * P + pos) * 4;
  f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
  if (i < len) {
    int s = sl;
    for (; s + (WG_RCH - 1) * S < splits; s += WG_RCH * S) {
      f32x4_t v[WG_RCH];
#pragma unroll
      for (int j = 0; j < WG_RCH; ++j) v[j] = *reinterpret_cast<const f32x4_t*>(ws + (long)(s + j * S) * len + i);
#pragma unroll
      for (int j = 0; j < WG_RCH; ++j) acc += v[j];
    }
    for (; s < splits; s += S) acc += *reinterpret_cast<const f32x4_t*>(ws + (long)s * len + i);
  }
  if constexpr (S > 1) {
    red[sl][pos] = acc;
    __syncthreads();
    if (sl != 0) return;
#pragma unroll
    for (int k = 1; k < S; ++k) acc += red[k][pos];
  }
  if (i >= len) return;
  f32x4_t d = *reinterpret_cast<const f32x4_t*>(dw + i);
  *reinterpret_cast<f32x4_t*>(dw + i) = d + scale * acc;
}

// split slices per position: enough workgroups (~512) for the chip when the weight is small
void launch_wgrad_splits_reduce(const float* ws, int splits, long len, float* dw, float scale, hipStream_t s) {
  const long n4 = (len + 3) / 4;
  int S = 1;
  while (S < 16 && S * 2 <= splits && (n4 * S) / 256 < 512) S *= 2;
  const unsigned grid = (unsigned)((n4 + 256 / S - 1) / (256 / S));
  switch (S) {
    case 1: hipLaunchKernelGGL(wgrad_splits_reduce_kernel<1>, dim3(grid), dim3(256), 0, s, ws, splits, len, dw, scale); break;
    case 2: hipLaunchKernelGGL(wgrad_splits_reduce_kernel<2>, dim3(grid), dim3(256), 0, s, ws, splits, len, dw, scale); break;
    case 4: hipLaunchKernelGGL(wgrad_splits_reduce_kernel<4>, dim3(grid), dim3(256), 0, s, ws, splits, len, dw, scale); break;
    case 8: hipLaunchKernelGGL(wgrad_splits_reduce_kernel<8>, dim3(grid), dim3(256), 0, s, ws, splits, len, dw, scale); break;
    default: hipLaunchKernelGGL(wgrad_splits_reduce_kernel<16>, dim3(grid), dim3(256), 0, s, ws, splits, len, dw, scale); break;
  }
}

// ------------------------------------------------- BatchNorm partial-statistics reduction
// Tile t carries (K_t, s_t = sum (y - K_t), q_t = sum (y - K_t)^2) over its n_t rows; moving to
// another shift K:  s = s_t + n_t d,  q = q_t + 2 d s_t + n_t d^2  with d = K_t - K.  Stage 1 folds
// chunks of BN_TCH tiles onto the chunk's first K, stage 2 folds the chunks onto row 0's value
// (the shift bn_apply reads back from y) and adds (sum, sumsq) into stats[2][N].  Fixed order.
constexpr int BN_TCH = 64;

__device__ __forceinline__ void shift_fold(float Kt, float st, float qt, float nt, float K, float& S, float& Q) {
  bn_shift_fold(Kt, st, qt, nt, K, S, Q);
}

// Both stages in ONE launch (grid (ceil(N/64), P)): block (g, p) folds tiles [64p, 64p+64) of channel
// group g onto the chunk's first K and leaves the chunk partial [P][3][N] in write-through (sc1)
// stores; per channel group the last block to arrive (relaxed agent-scope ticket, no release fence -
// the split-K hand-off of gemm_dense.h) acquires once and folds the P chunks in chunk order (the
// result does not depend on arrival order) into stats.  ctr: one zeroed uint32 per channel group,
// reset by its last arriver.  (Round 3 had stage 1 and stage 2 as two launches: one launch and one
// dependent boundary more per convolution with BN statistics.)
__global__ __launch_bounds__(256) void bn_part_fold(const float* __restrict__ part, int tiles, int N, long Mp, int BMr,
                                                    float* chunk, uint32_t* ctr, float* __restrict__ stats) {
  __shared__ float red[4][2][64];
  const int cl = threadIdx.x & 63, ln = threadIdx.x >> 6, c = blockIdx.x * 64 + cl, p = blockIdx.y;
  const int t0 = p * BN_TCH, t1 = min(tiles, t0 + BN_TCH);
  {
    float S = 0.f, Q = 0.f, K = 0.f;
    if (c < N) {
      K = part[(long)t0 * 3 * N + c];
      constexpr int PT = BN_TCH / 4;
      float kt[PT], st[PT], qt[PT];
#pragma unroll
      for (int i = 0; i < PT; ++i) {
        const int t = t0 + ln + 4 * i;
        const float* pt = part + (long)(t < t1 ? t : t0) * 3 * N + c;
        kt[i] = pt[0];
        st[i] = pt[N];
        qt[i] = pt[2 * N];
      }
#pragma unroll
      for (int i = 0; i < PT; ++i) {
        const int t = t0 + ln + 4 * i;
        if (t < t1) shift_fold(kt[i], st[i], qt[i], (float)min((long)BMr, Mp - (long)t * BMr), K, S, Q);
      }
    }
    red[ln][0][cl] = S;
    red[ln][1][cl] = Q;
    __syncthreads();
    if (ln == 0 && c < N) {
      S = ((red[0][0][cl] + red[1][0][cl]) + red[2][0][cl]) + red[3][0][cl];
      Q = ((red[0][1][cl] + red[1][1][cl]) + red[2][1][cl]) + red[3][1][cl];
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(chunk + (long)p * 3 * N, (short)0, 3 * N * 4,
                                                                          0x00020000);
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(K), rs, c * 4, 0, 16);
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(S), rs, (N + c) * 4, 0, 16);
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(Q), rs, (2 * N + c) * 4, 0, 16);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t prev = __hip_atomic_fetch_add(ctr + blockIdx.x, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const bool last = prev == gridDim.y - 1;
    if (last) {
      __hip_atomic_store(ctr + blockIdx.x, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // next launch / replay
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    red[0][0][0] = last ? 1.f : 0.f;
  }
  __syncthreads();
  const bool last = red[0][0][0] != 0.f;
  __syncthreads();
  if (!last) return;
  // stage 2 for this channel group (bn_part_stage2's fold)
  const int P = gridDim.y;
  float S = 0.f, Q = 0.f;
  if (c < N) {
    const float K = chunk[c];
    const long rows_chunk = (long)BN_TCH * BMr;
    for (int p0 = ln; p0 < P; p0 += 4 * 8) {
      float kp[8], sp[8], qp[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int pp = p0 + 4 * i;
        const float* pc = chunk + (long)(pp < P ? pp : 0) * 3 * N + c;
        kp[i] = pc[0];
        sp[i] = pc[N];
        qp[i] = pc[2 * N];
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int pp = p0 + 4 * i;
        if (pp < P) shift_fold(kp[i], sp[i], qp[i], (float)min(rows_chunk, Mp - (long)pp * rows_chunk), K, S, Q);
      }
    }
  }
  red[ln][0][cl] = S;
  red[ln][1][cl] = Q;
  __syncthreads();
  if (ln == 0 && c < N) {
    stats[c] += ((red[0][0][cl] + red[1][0][cl]) + red[2][0][cl]) + red[3][0][cl];
    stats[N + c] += ((red[0][1][cl] + red[1][1][cl]) + red[2][1][cl]) + red[3][1][cl];
  }
}

// ------------------------------------------------------------ host helpers
struct DevScratch {
  void* zeros = nullptr;
  void* ws = nullptr;
  size_t ws_bytes = 0;
};
std::mutex g_mu;
DevScratch g_dev[64];

const bf16* zero_page(hipStream_t s) {
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::lock_guard<std::mutex> lk(g_mu);
  DevScratch& d = g_dev[dev];
  if (!d.zeros) {
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    (void)hipStreamIsCapturing(s, &st);
    if (st != hipStreamCaptureStatusNone) throw std::runtime_error("igemm: first use inside a graph capture");
    if (hipMalloc(&d.zeros, 4096) != hipSuccess) throw std::runtime_error("igemm: zero page alloc");
    if (hipMemset(d.zeros, 0, 4096) != hipSuccess) throw std::runtime_error("igemm: zero page memset");
  }
  return reinterpret_cast<const bf16*>(d.zeros);
}

// Weight-gradient partial slabs live in their own buffer: the ResNet backward runs the weight
// gradients on a side stream, concurrently with the forward/data-gradient split-K launches.
DevScratch g_wg[64];

float* workspace(size_t bytes, hipStream_t s, DevScratch* pool = g_dev) {
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::lock_guard<std::mutex> lk(g_mu);
  DevScratch& d = pool[dev];
  if (d.ws_bytes < bytes) {
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    (void)hipStreamIsCapturing(s, &st);
    if (st != hipStreamCaptureStatusNone)
      throw std::runtime_error("igemm: workspace growth inside a graph capture (run the step eagerly first)");
    if (d.ws) {
      (void)hipStreamSynchronize(s);
      (void)hipFree(d.ws);
    }
    const size_t nb = std::max(bytes, d.ws_bytes * 3 / 2);
    if (hipMalloc(&d.ws, nb) != hipSuccess) throw std::runtime_error("igemm: workspace alloc");
    d.ws_bytes = nb;
  }
  return reinterpret_cast<float*>(d.ws);
}

DevScratch g_bn[64];
// the BN partial workspace starts with BN_CTR_BYTES of hand-off counters (bn_part_fold), zeroed at
// allocation and left zero by every launch; the partials follow
constexpr size_t BN_CTR_BYTES = 256;

float* bn_workspace(size_t bytes, hipStream_t s) {
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::lock_guard<std::mutex> lk(g_mu);
  DevScratch& d = g_bn[dev];
  bytes += BN_CTR_BYTES;
  if (d.ws_bytes < bytes) {
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    (void)hipStreamIsCapturing(s, &st);
    if (st != hipStreamCaptureStatusNone)
      throw std::runtime_error("igemm: BN partial workspace growth inside a graph capture (run the step eagerly first)");
    if (d.ws) {
      (void)hipStreamSynchronize(s);
      (void)hipFree(d.ws);
    }
    const size_t nb = std::max(bytes, d.ws_bytes * 3 / 2);
    if (hipMalloc(&d.ws, nb) != hipSuccess) throw std::runtime_error("igemm: BN partial workspace alloc");
    if (hipMemset(d.ws, 0, BN_CTR_BYTES) != hipSuccess) throw std::runtime_error("igemm: BN counter memset");
    d.ws_bytes = nb;
  }
  return reinterpret_cast<float*>(reinterpret_cast<char*>(d.ws) + BN_CTR_BYTES);
}

// the hand-off counters of the partials returned by bn_workspace (same device)
uint32_t* bn_counters(const float* part) {
  return reinterpret_cast<uint32_t*>(const_cast<char*>(reinterpret_cast<const char*>(part) - BN_CTR_BYTES));
}

void launch_bn_fold(float* part, int tiles, int N, long Mp, int BMr, float* stats, hipStream_t s) {
  const int nchunk = (tiles + BN_TCH - 1) / BN_TCH;
  float* chunk = part + (size_t)tiles * 3 * N;
  const unsigned cg = (unsigned)((N + 63) / 64);
  if (cg * sizeof(uint32_t) > BN_CTR_BYTES) throw std::runtime_error("bn_part_fold: too many channel groups");
  hipLaunchKernelGGL(bn_part_fold, dim3(cg, nchunk), dim3(256), 0, s, part, tiles, N, Mp, BMr, chunk, bn_counters(part),
                     stats);
}

int env_int(const char* name, int dflt) {
  const char* v = std::getenv(name);
  return v && *v ? std::atoi(v) : dflt;
}

struct Tile { int bm, bn; };

// Largest tile that still gives >= ~one workgroup per CU; DTFE_IG_TILE=BMxBN overrides.
// (An 8-wave 256-row-tile kernel with 3 LDS stages, one workgroup per CU, measured slower than
// these 4-wave tiles at two workgroups per CU on every ResNet-50 layer: profiles/r3_igemm_8wave_ab.txt.)
Tile pick_tile(long M, int N, int nphase) {
  const char* e = std::getenv("DTFE_IG_TILE");
  if (e && *e) {
    int bm = 0, bn = 0;
    if (std::sscanf(e, "%dx%d", &bm, &bn) == 2 && (bm == 64 || bm == 128) && (bn == 64 || bn == 128) && N % bn == 0)
      return {bm, bn};
  }
  constexpr long min_blocks = 240;
  const Tile cands[3] = {{128, 128}, {128, 64}, {64, 64}};
  for (const Tile& t : cands) {
    if (N % t.bn) continue;
    const long blocks = ((M + t.bm - 1) / t.bm) * (N / t.bn) * nphase;
    if (blocks >= min_blocks) return t;
  }
  return {64, 64};
}

template <int BM, int BN>
void launch_ig(IgemmArgs& a, long Mmax, hipStream_t s) {
  a.tiles_m = (int)((Mmax + BM - 1) / BM);
  dim3 grid(a.tiles_m * (a.N / BN), a.splits, a.nphase);
  // (a 32-deep-k-tile, 4-stage ring variant in the same 64 KB measured 12 % slower per conv pass:
  // profiles/r4_igemm_kb32_ab.txt)
  int nk_max = 0;
  for (int p = 0; p < a.nphase; ++p) nk_max = std::max(nk_max, a.ph[p].ntaps * (a.SC / IG_BK));
  // (a 1-stage, 3-workgroups-per-CU instance for the one-k-tile 1x1 convs measured 15-25 % slower
  // than this one: profiles/r3_resnet50_b256_kernels.txt)
  (void)nk_max;
  // (round 5, measured and removed: 64 x 256 whole-row tiles for the one-k-tile 1x1 convs - 64 -> 256
  // forward 175-180 vs 164-166 us, its data gradient 170 vs 155 us at B=256 - and the forward BN
  // statistics summed from the accumulator registers instead of the staged tile - no faster with the
  // statistics, 9-13 us slower per launch without them: profiles/r5_igemm_epilogue_ab.txt)
  if (a.bb_x)
    hipLaunchKernelGGL((igemm_kernel<BM, BN, 2, true, 2>), grid, dim3(IG_THREADS), 0, s, a);
  else
    hipLaunchKernelGGL((igemm_kernel<BM, BN, 2, false, 2>), grid, dim3(IG_THREADS), 0, s, a);
}

// returns true when BatchNorm statistics into bn_stats were produced (fused epilogue partials)
bool run_igemm(IgemmArgs& a, hipStream_t s, float* bn_stats = nullptr) {
  long Mmax = 0;
  for (int p = 0; p < a.nphase; ++p) Mmax = std::max(Mmax, (long)a.B * a.ph[p].RH * a.ph[p].RW);
  a.zeros = zero_page(s);
  if (a.nphase == 1 && a.bb_x) {
    // one-phase data gradient: its BN-backward statistics run as the separate pass
    // (launch_dgrad_bn_bwd_stats) - the per-tile kernel's LDS epilogue for them measured slower
    // (profiles/r2_resnet50_bn_bwd_fuse_ab.txt)
    a.bb_x = nullptr;
    bn_stats = nullptr;
  }
  Tile t = pick_tile(Mmax, a.N, a.nphase);
  a.splits = 1;
  a.ws = nullptr;
  if (a.nphase == 1 && a.ostr == 1) {
    // split-K when even the smallest tile leaves CUs idle and the k-loop is long
    const long blocks = ((Mmax + t.bm - 1) / t.bm) * (a.N / t.bn);
    const int nk = a.ph[0].ntaps * (a.SC / IG_BK);
    int sp = env_int("DTFE_IG_SPLIT", 0);
    constexpr long ftarget = 200;  // split-K workgroup target (R50 sweep: 400 -> 200 saves 0.15 ms)
    if (sp <= 0) {
      sp = 1;
      while (blocks * sp < ftarget && nk / (sp * 2) >= 6) sp *= 2;
    }
    sp = std::max(1, std::min(sp, nk));
    if (sp > 1) {
      a.splits = sp;
      a.ws = workspace((size_t)sp * Mmax * a.N * sizeof(float), s);
    }
  }
  // forward: BN statistics of the output (one phase, no accumulation); data gradient (a.bb_x set by
  // the caller): BN-backward statistics of the final, accumulated output, any phase count
  const bool bwd_bn = a.bb_x != nullptr;
  const bool fuse_bn = bn_stats && a.splits == 1 && (bwd_bn || (a.nphase == 1 && !a.accum));
  if (!fuse_bn) a.bb_x = nullptr;
  const int tiles_m = (int)((Mmax + t.bm - 1) / t.bm);
  const int tiles_all = tiles_m * (bwd_bn ? a.nphase : 1), nchunk = (tiles_all + BN_TCH - 1) / BN_TCH;
  a.bn_part = nullptr;
  if (fuse_bn) a.bn_part = bn_workspace(((size_t)tiles_all + nchunk) * 3 * a.N * sizeof(float), s);
  if (t.bm == 128 && t.bn == 128) launch_ig<128, 128>(a, Mmax, s);
  else if (t.bm == 128 && t.bn == 64) launch_ig<128, 64>(a, Mmax, s);
  else if (t.bm == 64 && t.bn == 128) launch_ig<64, 128>(a, Mmax, s);
  else launch_ig<64, 64>(a, Mmax, s);
  if (a.splits > 1) {
    const long len = Mmax * a.N;
    hipLaunchKernelGGL(splitk_to_bf16_kernel, dim3((unsigned)((len / 4 + 255) / 256)), dim3(256), 0, s, a.ws,
                       a.splits, len, a.out, a.accum);
  }
  if (!fuse_bn) return false;
  // (backward partials carry a zero shift: the row counts passed here then do not enter the fold)
  (void)nchunk;
  launch_bn_fold(a.bn_part, tiles_all, a.N, Mmax, t.bm, bn_stats, s);
  return true;
}

}  // namespace

uint32_t* bn_part_counter(const float* part) { return bn_counters(part) + (BN_CTR_BYTES / 4 - 1); }

float* bn_part_buffer(long tiles, int N, hipStream_t s) {
  const long nchunk = (tiles + BN_TCH - 1) / BN_TCH;
  return bn_workspace(((size_t)tiles + nchunk) * 3 * N * sizeof(float), s);
}

void launch_bn_part_reduce(float* part, int tiles, int N, long Mp, int BMr, float* stats, hipStream_t s) {
  launch_bn_fold(part, tiles, N, Mp, BMr, stats, s);
}

bool launch_igemm_fwd(const ConvFwdArgs& f, hipStream_t s, bool* stats_done) {
  const ConvGeom& g = f.g;
  if (g.C % IG_BK || g.Cout % 64 || g.KH * g.KW > IG_MAX_TAPS || g.pool_order || f.bias || f.act != 0) return false;
  IgemmArgs a;
  std::memset(&a, 0, sizeof(a));
  a.src = f.x; a.w = f.w; a.out = f.y;
  a.B = g.B; a.SH = g.H; a.SW = g.W; a.SC = g.C;
  a.N = g.Cout; a.Ktot = g.KH * g.KW * g.C;
  a.istr = g.stride; a.OHf = g.OH; a.OWf = g.OW; a.ostr = 1;
  a.nphase = 1;
  IgPhase& P = a.ph[0];
  P.RH = g.OH; P.RW = g.OW; P.oy = P.ox = 0;
  P.ntaps = g.KH * g.KW;
  for (int kh = 0; kh < g.KH; ++kh)
    for (int kw = 0; kw < g.KW; ++kw) {
      const int t = kh * g.KW + kw;
      P.dy[t] = kh - g.pad; P.dx[t] = kw - g.pad; P.kt[t] = t;
    }
  const bool st = run_igemm(a, s, f.bn_stats);
  if (stats_done) *stats_done = st;
  return true;
}

bool launch_igemm_dgrad(const ConvDgradArgs& d, hipStream_t s) {
  const ConvGeom& g = d.g;
  if (g.Cout % IG_BK || g.C % 64 || g.KH * g.KW > IG_MAX_TAPS || g.stride > 2 || d.unpool || d.relu_mask) return false;
  IgemmArgs a;
  std::memset(&a, 0, sizeof(a));
  a.src = d.dy; a.w = d.wt; a.out = d.dx;
  a.B = g.B; a.SH = g.OH; a.SW = g.OW; a.SC = g.Cout;
  a.N = g.C; a.Ktot = g.KH * g.KW * g.Cout;
  a.istr = 1; a.OHf = g.H; a.OWf = g.W; a.ostr = g.stride;
  a.accum = d.accumulate;
  a.acc_src = d.acc_src;
  a.acc_mask = d.acc_mask;
  if (a.acc_src && (!a.accum || g.stride != 1 || !a.acc_mask))
    throw std::runtime_error("conv_dgrad: a masked accumulation source needs accumulate, stride 1 and its mask");
  if (d.bnb_stats && !d.bnb_ymask) {  // (a bit-mask source: the separate statistics pass)
    a.bb_x = d.bnb_x; a.bb_y = d.bnb_y; a.bb_mean = d.bnb_mean; a.bb_invstd = d.bnb_invstd;
    a.bb_gamma = d.bnb_gamma; a.bb_beta = d.bnb_beta; a.bb_act = d.bnb_act;
  }
  const int st = g.stride;
  a.nphase = st * st;
  for (int py = 0; py < st; ++py)
    for (int px = 0; px < st; ++px) {
      IgPhase& P = a.ph[py * st + px];
      P.oy = py; P.ox = px;
      P.RH = (g.H - py + st - 1) / st;
      P.RW = (g.W - px + st - 1) / st;
      P.ntaps = 0;
      // dX[i*s+py][j*s+px] += dY[i + (py+pad-kh)/s][j + (px+pad-kw)/s] . W[kh][kw]  for exact divisions
      for (int kh = 0; kh < g.KH; ++kh) {
        const int ty = py + g.pad - kh;
        if (((ty % st) + st) % st) continue;
        for (int kw = 0; kw < g.KW; ++kw) {
          const int tx = px + g.pad - kw;
          if (((tx % st) + st) % st) continue;
          P.dy[P.ntaps] = ty / st; P.dx[P.ntaps] = tx / st; P.kt[P.ntaps] = kh * g.KW + kw;
          ++P.ntaps;
        }
      }
    }
  // Accumulating into dx (a bottleneck's input gradient on top of its shortcut share), a phase no
  // tap reaches contributes nothing: drop it instead of re-reading and re-writing its pixels (3 of
  // the 4 phases of a 1x1 / stride-2 projection - 617 MB of dead traffic per step at the ResNet-50
  // 56x56 layer).  BN-backward statistics need every phase's pixels, so they keep all phases.
  if (a.accum && !d.bnb_stats) {
    int n = 0;
    for (int p = 0; p < a.nphase; ++p)
      if (a.ph[p].ntaps > 0) a.ph[n++] = a.ph[p];
    if (n == 0) return true;
    a.nphase = n;
  }
  const bool fused = run_igemm(a, s, d.bnb_ymask ? nullptr : d.bnb_stats);
  if (d.bnb_stats && !fused) launch_dgrad_bn_bwd_stats(d, s);
  return true;
}

// DTFE_IG_W3: 0 off, 1 every eligible shape, 2 (default) only 64->64: measured 218 -> 143 us at
// 56x56 (B=256), equal at 28x28 128->128, slower at 14x14 / 7x7 where the per-tap kernel's
// 128x128 tiles fill the chip (profiles/r3_resnet50_wgrad3_ab.txt)
static bool use_wgrad3(const ConvGeom& g) {
  const int m = env_int("DTFE_IG_W3", 2);
  return m == 1 || (m == 2 && g.C <= 64 && g.Cout <= 64);
}

bool launch_igemm_wgrad(const ConvWgradArgs& f, hipStream_t s) {
  const ConvGeom& g = f.g;
  if (g.C % 64 || g.Cout % 64 || f.db || g.pool_order) return false;
  IgWgradArgs a;
  std::memset(&a, 0, sizeof(a));
  a.dy = f.dz; a.x = f.x;
  a.B = g.B; a.H = g.H; a.W = g.W; a.C = g.C; a.OH = g.OH; a.OW = g.OW; a.Cout = g.Cout;
  a.KH = g.KH; a.KW = g.KW; a.stride = g.stride; a.pad = g.pad;
  a.zeros = zero_page(s);
  if (g.KH == 3 && g.KW == 3 && g.stride == 1 && g.pad == 1 && g.OH == g.H && g.OW == g.W && g.W <= 62 &&
      (64 / g.W + 2) * (g.W + 2) <= W3_PATCH && use_wgrad3(g)) {
    // all 9 taps per workgroup from one staged patch (igemm_wgrad3_kernel)
    const int R = 64 / g.W;
    const int kpi = (g.H + R - 1) / R;
    const long tiles = (long)(g.Cout / 64) * (g.C / 64);
    const long T = (long)g.B * kpi;
    const long len = (long)g.Cout * 9 * g.C;
    // one workgroup per CU (the 36 accumulator tiles take the whole register file): aim for 192
    // workgroups (fewer than the CUs - the data-gradient chain keeps some), at least 4 k-tiles
    // each, fp32 partial slabs up to 40 MB
    constexpr long target = 192;  // (256 before round 4's side-stream sweep: 21.66-21.75 vs 21.76-21.81 ms,
                                  // profiles/r4_resnet50_wgrad_target_sweep.txt)
    long sp = env_int("DTFE_IG_WSPLIT", 0);
    if (sp <= 0) {
      sp = std::max(1L, std::min((target + tiles - 1) / tiles, T / 4));
      sp = std::max(1L, std::min(sp, (40L << 20) / (len * 4)));
    }
    sp = std::min(sp, T);
    a.splits = (int)sp;
    if (sp > 1) a.ws = workspace((size_t)sp * len * sizeof(float), s, g_wg);
    hipLaunchKernelGGL(igemm_wgrad3_kernel, dim3((unsigned)tiles, (unsigned)sp), dim3(IG_THREADS), 0, s, a, f.dw,
                       f.scale, R, kpi);
    if (sp > 1)
      launch_wgrad_splits_reduce(a.ws, (int)sp, len, f.dw, f.scale, s);
    return true;
  }
  const int bm = g.Cout % 128 == 0 ? 128 : 64, bn = g.C % 128 == 0 ? 128 : 64;
  const long tiles = (long)(g.Cout / bm) * g.KH * g.KW * (g.C / bn);
  const long M = (long)g.B * g.OH * g.OW;
  int sp = env_int("DTFE_IG_WSPLIT", 0);
  // splits: enough workgroups to fill the chip (target), each split at least 256 rows, and the
  // fp32 partial slabs (splits x weight size, written once and re-read by the reduce) bounded by
  // part_mb.  ResNet-50 B=256 sweeps: round 2 (profiles/r2_resnet50_wgrad_splits_ab.txt) 768 WGs /
  // unbounded 27.8 ms -> 512 WGs / 32 MB 27.0 ms per step; round 4, with the weight gradients on
  // their side stream beside the data-gradient chain (profiles/r4_resnet50_wgrad_target_sweep.txt):
  // 192 WGs 21.86-21.96 vs 512 22.31-22.35 ms (fewer partial slabs to write and reduce, and CUs
  // left to the main chain)
  constexpr long target = 192, part_mb = 32;
  if (sp <= 0) {
    sp = (int)std::max(1L, std::min((target + tiles - 1) / tiles, (M + 255) / 256));
    const long len0 = (long)g.Cout * g.KH * g.KW * g.C;
    sp = (int)std::max(1L, std::min((long)sp, (part_mb << 20) / (len0 * 4)));
  }
  long mchunk = (M + sp - 1) / sp;
  mchunk = (mchunk + 63) / 64 * 64;
  sp = (int)((M + mchunk - 1) / mchunk);
  a.splits = sp;
  a.mchunk = (int)mchunk;
  const long len = (long)g.Cout * g.KH * g.KW * g.C;
  if (sp > 1) a.ws = workspace((size_t)sp * len * sizeof(float), s, g_wg);
  dim3 grid((unsigned)tiles, sp);
  // 32-pixel k-tiles in a 4-stage ring (3 in flight, 2 WGs per CU); the 64-pixel 2- and 3-stage
  // rings measured slower (profiles/r4_igemm_kb32_ab.txt, scripts/archive/gpu_r4_wpipe.sh)
  if (bm == 128 && bn == 128)
    hipLaunchKernelGGL((igemm_wgrad_kernel<128, 128, 32, 4, 2>), grid, dim3(IG_THREADS), 0, s, a, f.dw, f.scale);
  else if (bm == 128)
    hipLaunchKernelGGL((igemm_wgrad_kernel<128, 64, 32, 4, 2>), grid, dim3(IG_THREADS), 0, s, a, f.dw, f.scale);
  else if (bn == 128)
    hipLaunchKernelGGL((igemm_wgrad_kernel<64, 128, 32, 4, 2>), grid, dim3(IG_THREADS), 0, s, a, f.dw, f.scale);
  else
    hipLaunchKernelGGL((igemm_wgrad_kernel<64, 64, 32, 4, 2>), grid, dim3(IG_THREADS), 0, s, a, f.dw, f.scale);
  if (sp > 1)
    launch_wgrad_splits_reduce(a.ws, sp, len, f.dw, f.scale, s);
  return true;
}

}  // namespace dtfe
