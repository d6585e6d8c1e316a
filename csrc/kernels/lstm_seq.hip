// Persistent whole-sequence LSTM kernels (TF BasicLSTMCell, LSTM:49-53).
//
// The reference unrolls 28 BasicLSTMCell steps (static_rnn): per step one [B,156]x[156,512]
// MatMul, a BiasAdd, split and four activations - dozens of launches per step.  Here ONE
// launch runs the whole forward recurrence and one the whole BPTT recurrence.  A workgroup
// owns 16 batch rows for all T steps (the recurrence only couples a row with itself, so no
// workgroup ever waits on another) and keeps everything the next step needs on-chip:
//
//   forward, per step t:  A = [x_t | h_{t-1}] (16 x 156, LDS; h written there by the
//     previous step's cell update) . K (156 x 512: each wave's 32-column slice is loaded once
//     into 78 VGPRs per lane and reused for all T steps) on exact-fp32 MFMA
//     (v_mfma_f32_16x16x4_f32, 16 waves x 32 gate columns) -> +bias, sigma/tanh (forget_bias folded in) -> gate tile in LDS -> cell
//     update c = c_prev * f + i * j, h = tanh(c) * o with c in registers.  act / c / h go to
//     HBM for the backward pass and the kernel-gradient GEMM.
//   backward, per step t = T-1..0: cell backward (dc carried in registers, dh from LDS) ->
//     dgates (LDS + HBM) -> dh_{t-1} = dgates . K_h^T (16 x 512 x 128 MFMA, k split over
//     two wave halves, partials summed through LDS; K_h^T fragments register-resident too).
//
// Gate order i, j, f, o and the formulas are those of the per-step kernels in
// elementwise.hip (lstm_cell_fwd / lstm_cell_bwd), which the tests compare against.
#include "lstm_seq.h"

#include "common.h"

namespace dtfe {

namespace {

constexpr int LR = 16;        // batch rows per workgroup (one MFMA row tile)
constexpr int LWAVES = 16;    // 1024 threads

template <int H, int KT4>
__global__ __launch_bounds__(1024) void lstm_seq_fwd_kernel(LstmSeqArgs a) {
  constexpr int G4 = 4 * H;
  constexpr int CPW = G4 / LWAVES;  // gate columns per wave
  constexpr int TPW = CPW / 16;     // 16-wide MFMA tiles per wave
  constexpr int GP = G4 + 4;        // gate tile pitch (floats)
  static_assert(CPW % 16 == 0, "H must be a multiple of 64");
  extern __shared__ float lds[];
  const int KT = a.I + H, AP = KT + 1;
  float* As = lds;            // [LR][AP]  [x_t | h_{t-1}]
  float* Gs = lds + LR * AP;  // [LR][GP]  activated gates
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r0 = blockIdx.x * LR, B = a.B;
  const long rowKT = KT;
  for (int e = tid; e < LR * KT; e += 1024) {
    const int r = e / KT, k = e - r * KT;
    As[r * AP + k] = a.xh[(long)(r0 + r) * rowKT + k];   // t = 0: x_0 and the initial h (zeros)
  }
  const int c0 = w * CPW, mrow = lane & 15, g = lane >> 4;
  // this wave's 32 gate columns of K as MFMA B fragments, loaded ONCE and kept in VGPRs for all
  // T steps (KT4 x TPW floats per lane): no per-step L2 traffic or load latency on the chain
  float kreg[KT4][TPW];
  {
    const float* kcol = a.K + c0 + mrow;
#pragma unroll
    for (int kk = 0; kk < KT4; ++kk)
#pragma unroll
      for (int j = 0; j < TPW; ++j) kreg[kk][j] = kcol[(long)(4 * kk + g) * G4 + 16 * j];
  }
  float creg[LR * H / 1024];
#pragma unroll
  for (int q = 0; q < LR * H / 1024; ++q) creg[q] = 0.f;
  // per-column gate bias (forget_bias folded in), hoisted out of the recurrence
  float bias_r[TPW];
#pragma unroll
  for (int j = 0; j < TPW; ++j) {
    const int col = c0 + 16 * j + mrow;
    bias_r[j] = a.bias[col] + (col / H == 2 ? a.forget_bias : 0.f);
  }
  // x_{t+1} does not depend on the recurrence: each thread prefetches its element (LR * I <= 1024,
  // checked at launch) right after step t's first barrier, so its HBM latency hides under step
  // t's MFMA + cell update instead of heading step t+1's critical path
  const bool xl = tid < LR * a.I;
  const int xr = xl ? tid / a.I : 0, xk = xl ? tid - xr * a.I : 0;
  float xnext = 0.f;
  for (int t = 0; t < a.T; ++t) {
    if (t > 0 && xl) As[xr * AP + xk] = xnext;
    __syncthreads();
    if (t + 1 < a.T && xl) xnext = a.xh[((long)(t + 1) * B + r0 + xr) * rowKT + xk];
    f32x4_t acc[TPW];
#pragma unroll
    for (int j = 0; j < TPW; ++j) acc[j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < KT4; ++kk) {
      const float av = As[mrow * AP + 4 * kk + g];
#pragma unroll
      for (int j = 0; j < TPW; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, kreg[kk][j], acc[j], 0, 0, 0);
    }
    float* act_t = a.act + ((long)t * B + r0) * G4;
#pragma unroll
    for (int j = 0; j < TPW; ++j) {
      const int col = c0 + 16 * j + mrow;
      const int gt = col / H;  // 0 i, 1 j, 2 f, 3 o
      const float bias = bias_r[j];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int r = 4 * g + e;
        const float z = acc[j][e] + bias;
        const float v = gt == 1 ? tanhf(z) : sigmoidf_(z);
        Gs[r * GP + col] = v;
        act_t[(long)r * G4 + col] = v;
      }
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < LR * H / 1024; ++q) {
      const int p = tid + 1024 * q, r = p / H, u = p - r * H;
      const float* gr = Gs + r * GP;
      const float si = gr[u], tj = gr[H + u], sf = gr[2 * H + u], so = gr[3 * H + u];
      const float c = creg[q] * sf + si * tj;
      creg[q] = c;
      const float h = tanhf(c) * so;
      a.c[((long)t * B + r0 + r) * H + u] = c;
      As[r * AP + a.I + u] = h;
      if (t + 1 < a.T) a.xh[((long)(t + 1) * B + r0 + r) * rowKT + a.I + u] = h;
      else a.hT[(long)(r0 + r) * H + u] = h;
    }
  }
}

template <int H>
__global__ __launch_bounds__(1024) void lstm_seq_bwd_kernel(LstmSeqArgs a) {
  constexpr int G4 = 4 * H;
  constexpr int GP = G4 + 4;   // dgate tile pitch (16 B aligned rows)
  constexpr int NT = H / 16;   // dh output tiles
  constexpr int KH = G4 / 2;   // k range per wave half
  static_assert(NT * 2 <= LWAVES, "H too large for one workgroup");
  extern __shared__ float lds[];
  float* DG = lds;                 // [LR][GP]
  float* P0 = DG + LR * GP;        // [LR][H] dh partial, k half 0
  float* P1 = P0 + LR * H;         // [LR][H] dh partial, k half 1
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r0 = blockIdx.x * LR, B = a.B;
  const int KT = a.I + H;
  // dh_{T-1} comes from the output layer
  for (int e = tid; e < LR * H; e += 1024) {
    P0[e] = a.dhT[(long)(r0 + e / H) * H + (e % H)];
    P1[e] = 0.f;
  }
  float dcreg[LR * H / 1024];
#pragma unroll
  for (int q = 0; q < LR * H / 1024; ++q) dcreg[q] = 0.f;
  __syncthreads();
  const int tile = w % NT, half = w / NT, mrow = lane & 15, g = lane >> 4;
  // this wave's K_h^T fragments (16 hidden units x its k half) in VGPRs for all T steps
  f32x4_t kb[KH / 16];
  {
    const float* krow = a.K + (long)(a.I + tile * 16 + mrow) * G4 + half * KH;
#pragma unroll
    for (int q = 0; q < KH / 16; ++q) kb[q] = *reinterpret_cast<const f32x4_t*>(krow + 16 * q + 4 * g);
  }
  // step t's saved gates and cells do not depend on the recurrence: registers hold step t's
  // (i, j, f, o, c_t, c_{t-1}) and step t-1's are loaded as soon as step t has read them, so
  // their HBM latency hides under step t's dgate stores and dh MFMA
  constexpr int NQ = LR * H / 1024;
  float pa[NQ][4], pc[NQ], pcp[NQ];
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const int p = tid + 1024 * q, r = p / H, u = p - r * H;
    const int t = a.T - 1;
    const float* ac = a.act + ((long)t * B + r0 + r) * G4;
#pragma unroll
    for (int gi = 0; gi < 4; ++gi) pa[q][gi] = ac[gi * H + u];
    const long ci = ((long)t * B + r0 + r) * H + u;
    pc[q] = a.c[ci];
    pcp[q] = t > 0 ? a.c[ci - (long)B * H] : 0.f;
  }
  for (int t = a.T - 1; t >= 0; --t) {
    float* dg_t = a.dg + ((long)t * B + r0) * G4;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int p = tid + 1024 * q, r = p / H, u = p - r * H;
      const float si = pa[q][0], tj = pa[q][1], sf = pa[q][2], so = pa[q][3];
      const float c = pc[q], cp = pcp[q];
      if (t > 0) {  // prefetch step t-1
        const float* an = a.act + ((long)(t - 1) * B + r0 + r) * G4;
#pragma unroll
        for (int gi = 0; gi < 4; ++gi) pa[q][gi] = an[gi * H + u];
        pc[q] = cp;
        pcp[q] = t > 1 ? a.c[((long)(t - 2) * B + r0 + r) * H + u] : 0.f;
      }
      const float dh = P0[r * H + u] + P1[r * H + u];
      const float tc = tanhf(c);
      const float dc = dcreg[q] + dh * so * (1.f - tc * tc);
      const float d0 = dc * tj * si * (1.f - si);
      const float d1 = dc * si * (1.f - tj * tj);
      const float d2 = dc * cp * sf * (1.f - sf);
      const float d3 = dh * tc * so * (1.f - so);
      dcreg[q] = dc * sf;
      float* dr = DG + r * GP;
      dr[u] = d0; dr[H + u] = d1; dr[2 * H + u] = d2; dr[3 * H + u] = d3;
      float* dgr = dg_t + (long)r * G4;
      dgr[u] = d0; dgr[H + u] = d1; dgr[2 * H + u] = d2; dgr[3 * H + u] = d3;
    }
    __syncthreads();
    if (t > 0 && half < 2) {
      // dh_{t-1}[r][u] = sum_c DG[r][c] * K[I + u][c]; lane group g supplies k = kb + 16q + 4g + e
      const float* drow = DG + mrow * GP + half * KH;
      f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int q = 0; q < KH / 16; ++q) {
        const f32x4_t av = *reinterpret_cast<const f32x4_t*>(drow + 16 * q + 4 * g);
#pragma unroll
        for (int e = 0; e < 4; ++e) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[e], kb[q][e], acc, 0, 0, 0);
      }
      float* P = half == 0 ? P0 : P1;
#pragma unroll
      for (int e = 0; e < 4; ++e) P[(4 * g + e) * H + tile * 16 + mrow] = acc[e];
    }
    __syncthreads();
  }
  (void)KT;
}

}  // namespace

bool launch_lstm_seq_fwd(const LstmSeqArgs& a, hipStream_t s) {
  // register-resident K slice: instantiated for the MNIST row-LSTM (I = 28, H = 128)
  if (a.H != 128 || a.I != 28 || a.B % LR || LR * a.I > 1024) return false;
  const size_t lds = ((size_t)LR * (a.I + a.H + 1) + (size_t)LR * (4 * a.H + 4)) * sizeof(float);
  auto k = lstm_seq_fwd_kernel<128, (28 + 128) / 4>;
  (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(k, dim3(a.B / LR), dim3(1024), lds, s, a);
  return true;
}

bool launch_lstm_seq_bwd(const LstmSeqArgs& a, hipStream_t s) {
  if (a.H != 128 || a.B % LR || (a.I + a.H) % 4) return false;
  const size_t lds = ((size_t)LR * (4 * a.H + 4) + 2 * (size_t)LR * a.H) * sizeof(float);
  auto k = lstm_seq_bwd_kernel<128>;
  (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(k, dim3(a.B / LR), dim3(1024), lds, s, a);
  return true;
}

}  // namespace dtfe
