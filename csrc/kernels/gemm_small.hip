// Latency-shaped exact-fp32 GEMM for the reference workloads' small dense layers (GAN,
// autoencoder: M, N <= ~800, K <= ~800 at batch 128 / 256).
//
// rocprof of those steps (profiles/r1_ref_gan_b128_trace.txt): every layer GEMM took 9-10 us on
// the LDS-staged 32x32 tile engine - 64-deep k-tiles each exposing an L2 round trip, plus the
// split-K hand-off (agent release / acquire fences) that auto split-K used to reach 256
// workgroups.  The work itself is < 1 us of v_mfma_f32_16x16x4_f32 per workgroup.  Here:
//
//  * one workgroup per 16 x 16 output tile (the tile grid alone reaches 128-833 workgroups for
//    these layers), its 4 waves splitting K four ways: no cross-workgroup reduction, no fences;
//  * every operand element of a wave's K slice is loaded straight from global memory into
//    MFMA fragment registers, all loads issued before the first MFMA (one memory latency per
//    16-group chunk, not one per k-tile), no LDS staging;
//  * the 4 k values a lane feeds into the 4 MFMAs of a 16-deep group are 4 CONSECUTIVE k
//    (lane group g = lane >> 4 holds k0 + 4g + j for MFMA j): a k-contiguous operand (KMAJ)
//    is one 16-byte load per group, a row-contiguous one (RMAJ) four 4-byte loads that 16
//    lanes read as one 64-byte segment.  A and B use the same k permutation, so the dot
//    product is unchanged;
//  * the 4 wave partials meet in LDS and are summed in wave order (bitwise reproducible), then
//    the shared dense epilogue (bias / activation / act' of aux / ones-row bias gradients /
//    dropout / beta / second output) runs one element per thread.
#include "gemm_dense.h"

namespace dtfe {

namespace {

constexpr int SG_CHUNK = 16;  // 16-deep k groups per register chunk (16 x 8 = 128 VGPRs of operands)

// 4 consecutive-k operand values of row r (A: m, B: n) at k = kb..kb+3 (zero past K / rows)
template <int MODE>
__device__ __forceinline__ f32x4_t load4(const float* p, long ld, int r, int rows, int ones_row, int kb, int K,
                                         bool vec) {
  f32x4_t v = {0.f, 0.f, 0.f, 0.f};
  if (r == ones_row) {
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = kb + j < K ? 1.f : 0.f;
    return v;
  }
  if (r >= rows) return v;
  if (MODE == KMAJ) {
    const float* q = p + (long)r * ld + kb;
    if (vec && kb + 4 <= K) return *reinterpret_cast<const f32x4_t*>(q);
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = kb + j < K ? q[j] : 0.f;
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = kb + j < K ? p[(long)(kb + j) * ld + r] : 0.f;
  }
  return v;
}

template <int AM, int BMD>
__global__ __launch_bounds__(256) void gemm_small_kernel(DenseGemmArgs a, int a_vec, int b_vec) {
  __shared__ float red[4][16][17];
  const int tiles_n = (a.N + 15) >> 4;
  const int tm = blockIdx.x / tiles_n, tn = blockIdx.x - tm * tiles_n;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = lane >> 4;
  const int m = tm * 16 + (lane & 15), n = tn * 16 + (lane & 15);
  // a ones row reads as 1.0 wherever it sits (load4 checks it before the memory read)
  const int a_rows = a.M, b_rows = a.N;
  const float* A = reinterpret_cast<const float*>(a.A);
  const float* B = reinterpret_cast<const float*>(a.B);
  // this wave's share of the 16-deep k groups
  const int G = (a.K + 15) >> 4;
  const int g0 = (G * w) >> 2, g1 = (G * (w + 1)) >> 2;
  f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
  for (int c0 = g0; c0 < g1; c0 += SG_CHUNK) {
    const int nc = min(SG_CHUNK, g1 - c0);
    f32x4_t fa[SG_CHUNK], fb[SG_CHUNK];
#pragma unroll
    for (int i = 0; i < SG_CHUNK; ++i) {
      if (i < nc) {
        const int kb = (c0 + i) * 16 + 4 * g;
        fa[i] = load4<AM>(A, a.lda, m, a_rows, a.a_ones_row, kb, a.K, a_vec);
        fb[i] = load4<BMD>(B, a.ldb, n, b_rows, a.b_ones_row, kb, a.K, b_vec);
      }
    }
#pragma unroll
    for (int i = 0; i < SG_CHUNK; ++i) {
      if (i < nc) {
#pragma unroll
        for (int j = 0; j < 4; ++j) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[i][j], fb[i][j], acc, 0, 0, 0);
      }
    }
  }
  // D: lane holds rows 4g..4g+3 (m), column lane & 15 (n)
#pragma unroll
  for (int j = 0; j < 4; ++j) red[w][4 * g + j][lane & 15] = acc[j];
  __syncthreads();
  const int r = threadIdx.x >> 4, c = threadIdx.x & 15;
  const int row = tm * 16 + r, col = tn * 16 + c;
  if (row >= a.M || col >= a.N) return;
  float x = ((red[0][r][c] + red[1][r][c]) + red[2][r][c]) + red[3][r][c];
  const int64_t drop_step = (a.keep < 1.f && a.counter) ? *a.counter : 0;
  if (!dense_epi(a, row, col, x, drop_step, 1.f / a.keep)) return;
  const long o = (long)row * a.ldc + col;
  if (a.out_f32) reinterpret_cast<float*>(a.out)[o] = x;
  else reinterpret_cast<bf16*>(a.out)[o] = f2bf(x);
}

}  // namespace

bool gemm_small_eligible(int dtype, const DenseGemmArgs& a) {
  // fp32 operands, fused epilogue only (no split-K / un-pool), a grid that is not huge
  const long tiles = (long)((a.M + 15) / 16) * ((a.N + 15) / 16);
  return dtype == 1 && !a.unpool && tiles <= 65535 && a.K >= 1;
}

void launch_gemm_small(int amode, int bmode, const DenseGemmArgs& a, hipStream_t s) {
  const int tiles = ((a.M + 15) / 16) * ((a.N + 15) / 16);
  const int a_vec = amode == KMAJ && a.lda % 4 == 0 && ((uintptr_t)a.A & 15) == 0;
  const int b_vec = bmode == KMAJ && a.ldb % 4 == 0 && ((uintptr_t)a.B & 15) == 0;
  auto go = [&](auto kern) { hipLaunchKernelGGL(kern, dim3(tiles), dim3(256), 0, s, a, a_vec, b_vec); };
  if (amode == KMAJ && bmode == KMAJ) go(gemm_small_kernel<KMAJ, KMAJ>);
  else if (amode == KMAJ && bmode == RMAJ) go(gemm_small_kernel<KMAJ, RMAJ>);
  else if (amode == RMAJ && bmode == KMAJ) go(gemm_small_kernel<RMAJ, KMAJ>);
  else go(gemm_small_kernel<RMAJ, RMAJ>);
}

}  // namespace dtfe
