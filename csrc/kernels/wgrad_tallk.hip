// Tall-K exact-fp32 weight gradient (SURVEY K03 for the LSTM, reference lstm/distributed_lstm.py:49-53:
// TF accumulates 28 per-step MatMul gradients of rnn/basic_lstm_cell/kernel).
//
//   out[m][n] = sum_k A[k*lda + m] * B[k*ldb + n]   (m < M, n < N)
//   bias[n]   = sum_k B[k*ldb + n]                  (the "ones row" m == M, optional)
//
// The LSTM kernel gradient is M = 156 ([x_t, h_{t-1}] columns), N = 512 gates, K = T*B = 3584 rows:
// a small output with a very long reduction.  The generic LDS-staged GEMM reached 80-320 workgroups
// and exposed one L2 round trip per 64-deep k-tile (34 us, rocprof).  Here the K range is split
// over `splits` workgroups per 64-column slab (8 x 32 = 256 workgroups), each owning the WHOLE
// (M+1) x 64 output of its K chunk: every operand element a workgroup loads is used by 16 MFMA
// columns (A) or all m-tiles of its wave (B), loads go straight into MFMA fragment registers
// (no LDS), and the next 8 k-steps' operands are in flight while the current ones multiply.
// Partial slabs [split][MP][N] are summed in split order by a second kernel (bitwise
// reproducible, no float atomics), which also stores (not accumulates) the gradient.
#include "common.h"
#include "lstm_seq.h"

#include <stdexcept>

namespace dtfe {

namespace {

constexpr int TK_BN = 64;   // output columns per workgroup (4 n-tiles of 16, shared by all waves)
constexpr int TK_KB = 8;    // k-steps (of 4 rows) per register batch

template <int MT>  // max m-tiles per wave (wave w owns m-tiles w, w+4, ...)
__global__ __launch_bounds__(256) void wgrad_tallk_kernel(TallKArgs a) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = lane >> 4, c = lane & 15;
  const int n0 = blockIdx.x * TK_BN;
  const int s = blockIdx.y;
  const int k0 = s * a.kchunk, k1 = min(a.K, k0 + a.kchunk);
  const int mtiles = (a.M + 1 + 15) >> 4;
  int mrow[MT];
  bool mval[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    const int mt = w + 4 * i;
    mval[i] = mt < mtiles;
    mrow[i] = mt * 16 + c;
  }
  f32x4_t acc[MT][4];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  float fa[2][TK_KB][MT], fb[2][TK_KB][4];
  auto load = [&](int buf, int kb0) {
#pragma unroll
    for (int q = 0; q < TK_KB; ++q) {
      const int k = kb0 + 4 * q + g;
      const bool kin = k < k1;
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        const int m = mrow[i];
        float v = 0.f;
        if (kin && mval[i]) v = m < a.M ? a.A[(long)k * a.lda + m] : (m == a.M && a.bias ? 1.f : 0.f);
        fa[buf][q][i] = v;
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[buf][q][j] = kin ? a.B[(long)k * a.ldb + n0 + j * 16 + c] : 0.f;
    }
  };
  auto mma = [&](int buf) {
#pragma unroll
    for (int q = 0; q < TK_KB; ++q)
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[buf][q][i], fb[buf][q][j], acc[i][j], 0, 0, 0);
  };
  // two register buffers, unrolled by two so every buffer index is a compile-time constant
  const int step = 4 * TK_KB;
  if (k0 < k1) load(0, k0);
  for (int kb = k0; kb < k1; kb += 2 * step) {
    if (kb + step < k1) load(1, kb + step);
    mma(0);
    if (kb + 2 * step < k1) load(0, kb + 2 * step);
    if (kb + step < k1) mma(1);
  }
  // lane holds rows 4g..4g+3 of each m-tile, column c of each n-tile
  float* part = a.ws + (long)s * a.MP * a.N;
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    if (!mval[i]) continue;
    const int mb = (w + 4 * i) * 16 + 4 * g;
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) part[(long)(mb + e) * a.N + n0 + j * 16 + c] = acc[i][j][e];
  }
}

__global__ __launch_bounds__(256) void tallk_reduce_kernel(TallKArgs a) {
  const long i = blockIdx.x * 256L + threadIdx.x;
  const int rows = a.M + (a.bias ? 1 : 0);
  if (i >= (long)rows * a.N) return;
  const int m = (int)(i / a.N), n = (int)(i - (long)m * a.N);
  const long stride = (long)a.MP * a.N;
  const float* p = a.ws + (long)m * a.N + n;
  float v[8];
  float t = 0.f;
  for (int s0 = 0; s0 < a.splits; s0 += 8) {
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] = s0 + q < a.splits ? p[(long)(s0 + q) * stride] : 0.f;
#pragma unroll
    for (int q = 0; q < 8; ++q) t += v[q];
  }
  t *= a.scale;
  if (m < a.M) a.out[(long)m * a.ldc + n] = t;
  else a.bias[n] = t;
}

}  // namespace

long tallk_ws_floats(int M, int N, int splits) { return (long)splits * (((M + 1 + 15) / 16) * 16) * N; }

void launch_wgrad_tallk(const TallKArgs& in, hipStream_t s) {
  TallKArgs a = in;
  if (a.N % TK_BN || a.M < 1 || a.K < 1 || a.splits < 1 || a.lda < a.M || a.ldb < a.N)
    throw std::runtime_error("wgrad_tallk: needs N % 64 == 0, lda >= M, ldb >= N, K >= 1, splits >= 1");
  const int mtiles = (a.M + 1 + 15) / 16;
  if (mtiles > 4 * 3) throw std::runtime_error("wgrad_tallk: M + 1 <= 192");
  a.MP = mtiles * 16;
  a.kchunk = ((a.K + a.splits - 1) / a.splits + 3) / 4 * 4;
  a.splits = (a.K + a.kchunk - 1) / a.kchunk;
  const dim3 grid(a.N / TK_BN, a.splits);
  if (mtiles <= 4) hipLaunchKernelGGL(wgrad_tallk_kernel<1>, grid, dim3(256), 0, s, a);
  else if (mtiles <= 8) hipLaunchKernelGGL(wgrad_tallk_kernel<2>, grid, dim3(256), 0, s, a);
  else hipLaunchKernelGGL(wgrad_tallk_kernel<3>, grid, dim3(256), 0, s, a);
  const long n = (long)(a.M + (a.bias ? 1 : 0)) * a.N;
  hipLaunchKernelGGL(tallk_reduce_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, a);
}

}  // namespace dtfe
