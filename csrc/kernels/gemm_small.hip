// Latency-shaped exact-fp32 GEMM for the reference workloads' small dense layers (GAN,
// autoencoder: M, N <= ~800, K <= ~800 at batch 128 / 256).
//
// rocprof of those steps (profiles/r1_ref_gan_b128_trace.txt): every layer GEMM took 9-10 us on
// the LDS-staged 32x32 tile engine - 64-deep k-tiles each exposing an L2 round trip, plus the
// split-K hand-off (agent release / acquire fences) that auto split-K used to reach 256
// workgroups.  The work itself is < 1 us of v_mfma_f32_16x16x4_f32 per workgroup.  Here:
//
//  * one workgroup per 16 x 16 output tile (the tile grid alone reaches 128-833 workgroups for
//    these layers), its 4 / 8 / 16 waves splitting K (by grid size): no cross-workgroup reduction, no fences;
//  * every operand element of a wave's K slice is loaded straight from global memory into
//    MFMA fragment registers, all loads issued before the first MFMA (one memory latency per
//    16-group chunk, not one per k-tile), no LDS staging;
//  * the 4 k values a lane feeds into the 4 MFMAs of a 16-deep group are 4 CONSECUTIVE k
//    (lane group g = lane >> 4 holds k0 + 4g + j for MFMA j): a k-contiguous operand (KMAJ)
//    is one 16-byte load per group, a row-contiguous one (RMAJ) four 4-byte loads that 16
//    lanes read as one 64-byte segment.  A and B use the same k permutation, so the dot
//    product is unchanged;
//  * the wave partials meet in LDS and are summed in wave order (bitwise reproducible), then
//    the shared dense epilogue (bias / activation / act' of aux / ones-row bias gradients /
//    dropout / beta / second output) runs one element per thread.
#include "gemm_dense.h"

#include <type_traits>

namespace dtfe {

namespace {


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

template <int AM, int BMD, int NW, int CH>
__device__ __forceinline__ void gemm_small_body(const DenseGemmArgs& a, int tile, int a_vec, int b_vec,
                                                float (*red)[16][17]) {
  const int tiles_n = (a.N + 15) >> 4;
  const int tm = tile / tiles_n, tn = tile - tm * tiles_n;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = lane >> 4;
  const int m = tm * 16 + (lane & 15), n = tn * 16 + (lane & 15);
  // a ones row reads as 1.0 wherever it sits (load4 checks it before the memory read)
  const int a_rows = a.M, b_rows = a.N;
  const float* A = reinterpret_cast<const float*>(a.A);
  const float* B = reinterpret_cast<const float*>(a.B);
  // this wave's share of the 16-deep k groups
  const int G = (a.K + 15) >> 4;
  const int g0 = (G * w) / NW, g1 = (G * (w + 1)) / NW;
  f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
  for (int c0 = g0; c0 < g1; c0 += CH) {
    const int nc = min(CH, g1 - c0);
    f32x4_t fa[CH], fb[CH];
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      if (i < nc) {
        const int kb = (c0 + i) * 16 + 4 * g;
        fa[i] = load4<AM>(A, a.lda, m, a_rows, a.a_ones_row, kb, a.K, a_vec);
        fb[i] = load4<BMD>(B, a.ldb, n, b_rows, a.b_ones_row, kb, a.K, b_vec);
      }
    }
#pragma unroll
    for (int i = 0; i < CH; ++i) {
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
  if (threadIdx.x >= 256) return;
  const int r = threadIdx.x >> 4, c = threadIdx.x & 15;
  const int row = tm * 16 + r, col = tn * 16 + c;
  if (row >= a.M || col >= a.N) return;
  float x = red[0][r][c];
#pragma unroll
  for (int i = 1; i < NW; ++i) x += red[i][r][c];  // wave order
  const int64_t drop_step = (a.keep < 1.f && a.counter) ? *a.counter : 0;
  if (!dense_epi(a, row, col, x, drop_step, 1.f / a.keep)) return;
  const long o = (long)row * a.ldc + col;
  if (a.out_f32) reinterpret_cast<float*>(a.out)[o] = x;
  else reinterpret_cast<bf16*>(a.out)[o] = f2bf(x);
}

template <int AM, int BMD, int NW, int CH>
__global__ __launch_bounds__(64 * NW) void gemm_small_kernel(DenseGemmArgs a, int a_vec, int b_vec) {
  __shared__ float red[NW][16][17];
  gemm_small_body<AM, BMD, NW, CH>(a, blockIdx.x, a_vec, b_vec, red);
}

// Two independent small GEMMs of one backward phase in ONE launch (a layer's weight gradient (RMAJ, RMAJ)
// beside its data gradient (KMAJ, KMAJ)): workgroups [0, t0) run the first, the rest the second - one
// dependent launch fewer per layer in the GAN / autoencoder steps, which are chains of ~5 us launches.
struct SmallPair {
  DenseGemmArgs g0, g1;
  int t0, v0a, v0b, v1a, v1b;
};
template <int NW, int CH>
__global__ __launch_bounds__(64 * NW) void gemm_small_pair_kernel(SmallPair p) {
  __shared__ float red[NW][16][17];
  if ((int)blockIdx.x < p.t0) gemm_small_body<RMAJ, RMAJ, NW, CH>(p.g0, blockIdx.x, p.v0a, p.v0b, red);
  else gemm_small_body<KMAJ, KMAJ, NW, CH>(p.g1, blockIdx.x - p.t0, p.v1a, p.v1b, red);
}
// 8-deep operand chunks (~90 VGPRs: 5 waves per SIMD); the 16-deep chunks of round 2 took 163 VGPRs
constexpr int SCH = 8;
// waves per tile by grid size: >= 512 tiles already give >= 2048 waves at a 4-way K split (fewer, longer
// waves, a 4-partial LDS reduce), >= 256 tiles take an 8-way split, smaller grids 16 ways.  Against 16
// everywhere: GAN 0.0697 -> 0.0624 ms, autoencoder 0.0806 -> 0.0721 (4 everywhere: 0.0674 / 0.0745; other
// thresholds in profiles/r6_ref_models_fused.txt)
int small_waves(long tiles) { return tiles >= 512 ? 4 : tiles >= 256 ? 8 : 16; }
template <typename F>
void by_waves(long tiles, F&& f) {
  const int nw = small_waves(tiles);
  if (nw == 4) f(std::integral_constant<int, 4>{});
  else if (nw == 8) f(std::integral_constant<int, 8>{});
  else f(std::integral_constant<int, 16>{});
}

int small_tiles(const DenseGemmArgs& a) { return ((a.M + 15) / 16) * ((a.N + 15) / 16); }
int small_vec(int mode, const void* p, int ld) { return mode == KMAJ && ld % 4 == 0 && ((uintptr_t)p & 15) == 0; }

}  // namespace

bool gemm_small_eligible(int dtype, const DenseGemmArgs& a) {
  // fp32 operands, fused epilogue only (no split-K / un-pool), a grid that is not huge
  const long tiles = (long)((a.M + 15) / 16) * ((a.N + 15) / 16);
  return dtype == 1 && !a.unpool && tiles <= 65535 && a.K >= 1;
}

void launch_gemm_small(int amode, int bmode, const DenseGemmArgs& a, hipStream_t s) {
  const int tiles = small_tiles(a);
  const int a_vec = small_vec(amode, a.A, a.lda), b_vec = small_vec(bmode, a.B, a.ldb);
  by_waves(tiles, [&](auto nwc) {
    constexpr int SW = decltype(nwc)::value;
    auto go = [&](auto kern) { hipLaunchKernelGGL(kern, dim3(tiles), dim3(64 * SW), 0, s, a, a_vec, b_vec); };
    if (amode == KMAJ && bmode == KMAJ) go(gemm_small_kernel<KMAJ, KMAJ, SW, SCH>);
    else if (amode == KMAJ && bmode == RMAJ) go(gemm_small_kernel<KMAJ, RMAJ, SW, SCH>);
    else if (amode == RMAJ && bmode == KMAJ) go(gemm_small_kernel<RMAJ, KMAJ, SW, SCH>);
    else go(gemm_small_kernel<RMAJ, RMAJ, SW, SCH>);
  });
}

void launch_gemm_small_group(int n, const int* am, const int* bm, const DenseGemmArgs* g, hipStream_t s) {
  int i0 = -1, i1 = -1;  // the (RMAJ, RMAJ) piece and the (KMAJ, KMAJ) piece
  for (int i = 0; i < n; ++i) {
    if (am[i] == RMAJ && bm[i] == RMAJ && i0 < 0) i0 = i;
    else if (am[i] == KMAJ && bm[i] == KMAJ && i1 < 0) i1 = i;
  }
  if (n != 2 || i0 < 0 || i1 < 0 || (long)small_tiles(g[0]) + small_tiles(g[1]) > 65535) {
    for (int i = 0; i < n; ++i) launch_gemm_small(am[i], bm[i], g[i], s);  // separate launches, recording order
    return;
  }
  SmallPair p;
  p.g0 = g[i0];
  p.g1 = g[i1];
  p.t0 = small_tiles(p.g0);
  p.v0a = small_vec(RMAJ, p.g0.A, p.g0.lda);
  p.v0b = small_vec(RMAJ, p.g0.B, p.g0.ldb);
  p.v1a = small_vec(KMAJ, p.g1.A, p.g1.lda);
  p.v1b = small_vec(KMAJ, p.g1.B, p.g1.ldb);
  const int grid = p.t0 + small_tiles(p.g1);
  by_waves(grid, [&](auto nwc) {
    constexpr int SW = decltype(nwc)::value;
    hipLaunchKernelGGL((gemm_small_pair_kernel<SW, SCH>), dim3(grid), dim3(64 * SW), 0, s, p);
  });
}

}  // namespace dtfe
