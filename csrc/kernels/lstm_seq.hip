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

#include <cstdlib>
#include <type_traits>

namespace dtfe {

namespace {

constexpr int LR = 16;        // batch rows per workgroup (one MFMA row tile)

// d loss / d h_T of (row, unit): given (dhT), or dl[row] . W_out[unit] (the fused head's dlogits)
__device__ __forceinline__ float dh_t_of(const LstmSeqArgs& a, int row, int u) {
  if (!a.dl) return a.dhT[(long)row * a.H + u];
  float s = 0.f;
  for (int c = 0; c < a.nc; ++c) s = __builtin_fmaf(a.dl[(long)row * a.nc + c], a.wo[(long)u * a.nc + c], s);
  return s;
}
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
    P0[e] = dh_t_of(a, r0 + e / H, e % H);
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

// ------------------------------------------------------------------ 4-way split recurrence
// The kernels above run each 16-row group on ONE CU, and the exact-fp32 MFMA (1/16 of the bf16
// rate) makes every timestep ~10k cycles of matrix work on that CU: 8 CUs busy, 248 idle.  Here
// each row group is split over NS = 4 workgroups (4 CUs) by HIDDEN UNIT: workgroup sp owns units
// [32 sp, 32 sp + 32) and therefore the 128 gate columns {i, j, f, o} x those units - so the cell
// update (which couples the four gates of a unit) stays inside the workgroup and a timestep does
// a quarter of the MFMA work.  The only coupling is the recurrent operand: the forward needs all
// 128 units of h_{t-1}, the backward all 512 dgate columns of step t.
//
// Exchange: a flag-per-word ("low latency") protocol.  Every exchanged fp32 travels as one 64-bit
// word {value, tag} stored with a single agent-scope atomic store, tag = epoch * 256 + step + 1
// (never 0, the zero-filled buffer's tag); the reader polls the words it needs with agent-scope
// atomic loads until every tag matches.  A
// separate flag would cost a second memory round trip and a release fence (L2 write-back on the
// multi-L2 gfx950) per step; here a step costs one store->load propagation.  Buffers are double
// (step parity): slot t&1 is rewritten at step t+2 only after its writer has read the step-t+1
// words of every peer, which those peers produce after they finished reading slot t&1.  The epoch
// (advanced by the last workgroup of each launch) makes stale words of earlier launches - and
// graph replays - never match, so nothing is reset between launches.  Polls are bounded by a
// wall-clock timeout that sets an error word instead of hanging.  All 4 * B/16 workgroups must
// be co-resident (one 512-thread workgroup per CU, <= 256): checked at launch.
// NS = 8 (round 6): 8 workgroups of 256 threads per row group, each owning 16 units - half the MFMA
// work per step and per CU (4 waves, one per SIMD) for the same exchange; used where the grid of
// B/16 x 8 workgroups fits (B <= 512), NS = 4 above that.
constexpr int NS_MAX = 8;
constexpr int MAX_GROUPS = 64;
template <int NS>
constexpr int split_threads() { return LR * 128 / NS; }  // one thread per (row, unit) of the slice (H = 128)

struct SplitSync {
  unsigned long long* llf;  // [MAX_GROUPS][2][16][H]   forward h exchange
  unsigned long long* llb;  // [MAX_GROUPS][2][NS][16][H] backward dh-partial exchange
  int* epoch;
  int* done;
  int* err;
};

__device__ __forceinline__ void ll_put(unsigned long long* p, float v, unsigned tag) {
  const unsigned long long w = ((unsigned long long)tag << 32) | __float_as_uint(v);
  __hip_atomic_store(p, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// N words per thread at p[k * stride]; returns when every tag equals `tag` (or on timeout)
template <int N>
__device__ __forceinline__ void ll_get(const unsigned long long* p, long stride, unsigned tag, float (&v)[N], int* err) {
  unsigned long long w[N];
#pragma unroll
  for (int k = 0; k < N; ++k) w[k] = __hip_atomic_load(p + k * stride, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  unsigned long long t0 = 0;
  for (;;) {
    bool ok = true;
#pragma unroll
    for (int k = 0; k < N; ++k) ok &= (unsigned)(w[k] >> 32) == tag;
    if (ok) break;
    if (!t0) t0 = wall_clock64();
    else if (wall_clock64() - t0 > 2000000000ull) {  // 20 s at 100 MHz: a peer never ran - fail, do not hang
      __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      break;
    }
#pragma unroll
    for (int k = 0; k < N; ++k)
      if ((unsigned)(w[k] >> 32) != tag) w[k] = __hip_atomic_load(p + k * stride, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
#pragma unroll
  for (int k = 0; k < N; ++k) v[k] = __uint_as_float((unsigned)w[k]);
}

__device__ __forceinline__ void finish_launch(const SplitSync& y) {
  __syncthreads();
  if (threadIdx.x == 0) {
    const int prev = __hip_atomic_fetch_add(y.done, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (prev == (int)gridDim.x - 1) {
      __hip_atomic_store(y.done, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add(y.epoch, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// (row group, split) of this workgroup.  Workgroups are dealt to the 8 XCDs round-robin by id, so
// with a multiple of 8 row groups the NS workgroups of one group - the ones that exchange h / dh
// every step - get ids rg, rg + G, ... and sit on ONE XCD (its L2); otherwise consecutive ids.
template <int NS>
__device__ __forceinline__ void split_coords(int groups, int& rg, int& sp) {
  if (groups % 8 == 0) {
    rg = blockIdx.x % groups;
    sp = blockIdx.x / groups;
  } else {
    rg = blockIdx.x / NS;
    sp = blockIdx.x % NS;
  }
}

__device__ __forceinline__ unsigned launch_base(const SplitSync& y) {
  return (unsigned)__hip_atomic_load(y.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) * 256u;
}

// forward: A = [x_t | h_{t-1}] (16 x 156, LDS) . K[:, my 128 gate columns] (each wave one 16-column
// tile, its 39 k-steps of B fragments in VGPRs for all T steps) on v_mfma_f32_16x16x4_f32.
template <int H, int KT4, int NS>
__global__ __launch_bounds__(LR * H / NS) void lstm_split_fwd_kernel(LstmSeqArgs a, SplitSync y) {
  constexpr int SPT = LR * H / NS;         // one thread per (row, unit) of the slice: 512 / 256
  constexpr int G4 = 4 * H, UPW = H / NS;  // units per workgroup (32 / 16)
  constexpr int GC = 4 * UPW;              // gate columns per workgroup (128 / 64) = one 16-wide tile per wave
  constexpr int GP = GC + 4;
  constexpr int HW = LR * H / SPT;         // exchanged h words per thread (NS)
  constexpr int TPG = UPW / 16;            // unit tiles per gate (2 / 1)
  static_assert(GC / 16 == SPT / 64, "one gate-column tile per wave");
  extern __shared__ float lds[];
  const int I = a.I, KT = I + H, AP = KT + 1;
  float* As = lds;            // [16][AP]
  float* Gs = lds + 16 * AP;  // [16][GP] activated gates of my columns (gate-major: gi * UPW + u)
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  int rg, sp;
  split_coords<NS>(a.B / LR, rg, sp);
  const int r0 = rg * LR, B = a.B;
  const unsigned base = launch_base(y);
  const long rowKT = KT;
  unsigned long long* llg = y.llf + (long)rg * 2 * LR * H;
  const int mrow = lane & 15, g = lane >> 4;
  // wave w: gate gi = w / TPG, units 16 * (w % TPG) .. +16 of my slice
  const int gi = w / TPG, ul = 16 * (w % TPG) + mrow, col = gi * H + sp * UPW + ul;  // global gate column
  float kreg[KT4];
#pragma unroll
  for (int kk = 0; kk < KT4; ++kk) kreg[kk] = a.K[(long)(4 * kk + g) * G4 + col];
  const float bias = a.bias[col] + (gi == 2 ? a.forget_bias : 0.f);
  // batch staging folded in (a.st.x: the images [B][T*I]): the recurrence reads x_t from the images, and
  // the NS workgroups of a row group share writing its x rows into xh (read only by the kernel gradient),
  // the labels and the accumulator clears - one launch and one pass over the batch fewer per step
  const bool staged = a.st.x != nullptr;
  const int TI = a.T * I;
  if (staged) {
    for (int e = sp * SPT + tid; e < LR * TI; e += NS * SPT) {
      const int r = e / TI, rem = e - r * TI, t = rem / I;
      a.xh[((long)t * B + r0 + r) * rowKT + rem - t * I] = a.st.x[(long)(r0 + r) * TI + rem];
    }
    const long yrow = a.st.ny / B;
    if (sp == 0)
      for (long e = tid; e < LR * yrow; e += SPT) a.st.ydst[r0 * yrow + e] = a.st.ysrc[r0 * yrow + e];
    if (blockIdx.x == 0)
      for (int z = 0; z < a.st.nz; ++z)
        for (long i = tid; i < a.st.zlen[z]; i += SPT) a.st.zptr[z][i] = 0u;
  }
  // cell update ownership: thread -> (row, unit) of my 16 x 32 slice
  const int cr = tid / UPW, cu = tid - cr * UPW;
  float creg = 0.f;
  // x_t: XPT elements per thread (LR * I = 448), prefetched a step ahead so their load latency is
  // off the recurrence's critical path
  constexpr int XPT = (LR * 28 + SPT - 1) / SPT;
  int xr[XPT], xk[XPT];
  bool xo[XPT];
  float xv[XPT];
  const float* xp[XPT];
  const long xstep = staged ? (long)I : (long)B * rowKT;  // x_t -> x_{t+1}
#pragma unroll
  for (int j = 0; j < XPT; ++j) {
    const int e = tid + j * SPT;
    xo[j] = e < LR * I;
    xr[j] = xo[j] ? e / I : 0;
    xk[j] = xo[j] ? e - xr[j] * I : 0;
    xp[j] = staged ? a.st.x + (long)(r0 + xr[j]) * TI + xk[j] : a.xh + ((long)r0 + xr[j]) * rowKT + xk[j];
    xv[j] = xo[j] ? xp[j][0] : 0.f;
  }
  for (int t = 0; t < a.T; ++t) {
#pragma unroll
    for (int j = 0; j < XPT; ++j) {
      if (xo[j]) As[xr[j] * AP + xk[j]] = xv[j];
      if (xo[j] && t + 1 < a.T) xv[j] = xp[j][(t + 1) * xstep];
    }
    if (t == 0) {
      for (int e = tid; e < LR * H; e += SPT) {
        const long o = ((long)r0 + e / H) * rowKT + I + e % H;
        As[(e / H) * AP + I + e % H] = staged ? 0.f : a.xh[o];  // h_{-1} = 0
        if (staged && sp == 0) a.xh[o] = 0.f;
      }
    } else {
      float hv[HW];
      ll_get<HW>(llg + ((t - 1) & 1) * LR * H + tid, SPT, base + t, hv, y.err);
#pragma unroll
      for (int k = 0; k < HW; ++k) {
        const int e = tid + k * SPT;
        As[(e / H) * AP + I + e % H] = hv[k];
      }
    }
    __syncthreads();
    f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < KT4; ++kk) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(As[mrow * AP + 4 * kk + g], kreg[kk], acc, 0, 0, 0);
    float* act_t = a.act + ((long)t * B + r0) * G4;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int r = 4 * g + e;
      const float z = acc[e] + bias;
      const float v = gi == 1 ? tanhf(z) : sigmoidf_(z);
      Gs[r * GP + gi * UPW + ul] = v;
      act_t[(long)r * G4 + col] = v;
    }
    __syncthreads();
    {
      const float* gr = Gs + cr * GP;
      const float si = gr[cu], tj = gr[UPW + cu], sf = gr[2 * UPW + cu], so = gr[3 * UPW + cu];
      const float c = creg * sf + si * tj;
      creg = c;
      const float h = tanhf(c) * so;
      const int u = sp * UPW + cu;
      a.c[((long)t * B + r0 + cr) * H + u] = c;
      if (t + 1 < a.T) {
        ll_put(llg + (t & 1) * LR * H + cr * H + u, h, base + t + 1);
        a.xh[((long)(t + 1) * B + r0 + cr) * rowKT + I + u] = h;  // for the kernel-gradient GEMM
      } else {
        a.hT[(long)(r0 + cr) * H + u] = h;
      }
    }
    // no barrier needed here: the next As writes come after this step's post-MFMA barrier, the
    // next Gs writes after the next step's post-exchange barrier (which every reader of Gs passes)
  }
  finish_launch(y);
}

// backward, per step t = T-1..0: cell backward of my 16 x 32 units (dh of my units from the
// exchange, dc in a register; act / c of the next step prefetched) -> my 128 dgate columns ->
// dg[t] and LDS; then this workgroup's PARTIAL dh_{t-1}[16][all 128 units] = dg_t[:, my columns]
// . K_h[:, my columns]^T (8 waves = 8 unit tiles, 32 k4-steps) goes to the exchange, and each
// thread sums the 4 partials of its (row, unit) in a fixed order - 4 words per thread per step
// instead of gathering all 512 dgate columns.
template <int H, int NS>
__global__ __launch_bounds__(LR * H / NS) void lstm_split_bwd_kernel(LstmSeqArgs a, SplitSync y) {
  constexpr int SPT = LR * H / NS;
  constexpr int G4 = 4 * H, UPW = H / NS, GC = 4 * UPW;  // my gate columns (128 / 64) = 32 / 16 k4-steps
  constexpr int DP = GC + 4;
  constexpr int TPW = (H / 16) / (SPT / 64);              // dh unit tiles per wave (1 / 2)
  extern __shared__ float lds[];
  float* DG = lds;  // [2][16][DP] my dgates of step t (parity-double-buffered: one barrier per step)
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  int rg, sp;
  split_coords<NS>(a.B / LR, rg, sp);
  const int r0 = rg * LR, B = a.B;
  const unsigned base = launch_base(y);
  unsigned long long* llg = y.llb + (long)rg * 2 * NS * LR * H;  // [2][NS src][16][H] (groups at NS_MAX pitch below)
  const int mrow = lane & 15, g = lane >> 4;
  // B fragments: B[k = j][n = u] = K[I + u][col(j)], j = my gate column q * UPW + v -> q * H + sp * UPW + v,
  // u = 16 (w TPW + tt) + mrow (wave w = unit tiles w TPW .. + TPW)
  float kb[TPW][GC / 4];
#pragma unroll
  for (int tt = 0; tt < TPW; ++tt) {
    const float* krow = a.K + (long)(a.I + 16 * (w * TPW + tt) + mrow) * G4 + sp * UPW;
#pragma unroll
    for (int kk = 0; kk < GC / 4; ++kk) {
      const int j = 4 * kk + g;
      kb[tt][kk] = krow[(j / UPW) * H + j % UPW];
    }
  }
  const int cr = tid / UPW, cu = tid - cr * UPW, u = sp * UPW + cu;
  float dh = dh_t_of(a, r0 + cr, u);
  float dc = 0.f;
  auto fetch = [&](int t, float (&v)[6]) {
    const long ri = (long)t * B + r0 + cr;
    const float* ac = a.act + ri * G4;
    v[0] = ac[u];
    v[1] = ac[H + u];
    v[2] = ac[2 * H + u];
    v[3] = ac[3 * H + u];
    v[4] = a.c[ri * H + u];
    v[5] = t > 0 ? a.c[(ri - B) * H + u] : 0.f;
  };
  float nx[6];
  fetch(a.T - 1, nx);
  for (int t = a.T - 1; t >= 0; --t) {
    const float si = nx[0], tj = nx[1], sf = nx[2], so = nx[3], c = nx[4], cp = nx[5];
    if (t > 0) fetch(t - 1, nx);
    float* D = DG + (t & 1) * 16 * DP;
    {
      const float tc = tanhf(c);
      const float dct = dc + dh * so * (1.f - tc * tc);
      const float d4[4] = {dct * tj * si * (1.f - si), dct * si * (1.f - tj * tj), dct * cp * sf * (1.f - sf),
                           dh * tc * so * (1.f - so)};
      float* dgr = a.dg + ((long)t * B + r0 + cr) * G4;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        dgr[q * H + u] = d4[q];
        D[cr * DP + q * UPW + cu] = d4[q];
      }
      dc = dct * sf;
    }
    if (t == 0) break;
    __syncthreads();
    f32x4_t acc[TPW];
#pragma unroll
    for (int tt = 0; tt < TPW; ++tt) acc[tt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    const float* drow = D + mrow * DP;
#pragma unroll
    for (int kk = 0; kk < GC / 4; ++kk) {
      const float av = drow[4 * kk + g];
#pragma unroll
      for (int tt = 0; tt < TPW; ++tt) acc[tt] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, kb[tt][kk], acc[tt], 0, 0, 0);
    }
    unsigned long long* slot = llg + (long)(t & 1) * NS * LR * H;
#pragma unroll
    for (int tt = 0; tt < TPW; ++tt)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        ll_put(slot + ((long)sp * LR + 4 * g + e) * H + 16 * (w * TPW + tt) + mrow, acc[tt][e], base + t + 1);
    float pv[NS];
    ll_get<NS>(slot + (long)cr * H + u, (long)LR * H, base + t + 1, pv, y.err);
    float s = pv[0];  // the NS partials in a fixed order
#pragma unroll
    for (int q = 1; q < NS; ++q) s += pv[q];
    dh = s;
  }
  finish_launch(y);
}

char* g_split_buf[64] = {};

SplitSync split_sync(hipStream_t s, int H) {
  char** buf = g_split_buf;
  constexpr size_t CTL = 4096;
  const size_t fw = (size_t)MAX_GROUPS * 2 * LR * 128, bw = fw * NS_MAX;  // words, H = 128
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (H != 128 || dev < 0 || dev >= 64) return SplitSync{};
  if (!buf[dev]) {
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    (void)hipStreamIsCapturing(s, &st);
    if (st != hipStreamCaptureStatusNone) return SplitSync{};  // first use inside a capture: fall back
    const size_t bytes = CTL + (fw + bw) * 8;
    char* p = nullptr;
    if (hipMalloc(&p, bytes) != hipSuccess) return SplitSync{};
    if (hipMemset(p, 0, bytes) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
      (void)hipFree(p);
      return SplitSync{};
    }
    buf[dev] = p;
  }
  int* c = reinterpret_cast<int*>(buf[dev]);
  auto* ll = reinterpret_cast<unsigned long long*>(buf[dev] + CTL);
  return SplitSync{ll, ll + fw, c, c + 4, c + 8};
}

// every workgroup of a split launch must be resident at once (they exchange h every step): the
// grid must fit the occupancy the runtime reports for this kernel and LDS size, times the CUs
bool co_resident(const void* kern, int threads, size_t lds, int blocks) {
  int dev = 0, per_cu = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess) return false;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return false;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, threads, lds) != hipSuccess) return false;
  return per_cu >= 1 && (long)per_cu * cus >= blocks;
}

// workgroups per row group of the split kernels: 0 = no split.  DTFE_LSTM_SPLIT (read per launch: tests A/B
// the paths in one process): 0 off, 4 / 8 force that split, unset / 1 = 8 where B/16 x 8 <= 256, else 4.
int split_ns(const LstmSeqArgs& a) {
  const char* e = getenv("DTFE_LSTM_SPLIT");
  const int v = e ? atoi(e) : 1;
  // one workgroup per CU, all co-resident: <= 256 workgroups; exchange buffers sized for MAX_GROUPS
  if (v == 0 || a.H != 128 || a.I != 28 || a.B % LR != 0 || a.B / LR > MAX_GROUPS || a.T >= 255) return 0;
  const int groups = a.B / LR;
  if (v != 4 && groups * 8 <= 256) return 8;
  return groups * 4 <= 256 ? 4 : 0;
}

}  // namespace

int lstm_split_status(bool reset) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64 || !g_split_buf[dev]) return 0;
  int* err = reinterpret_cast<int*>(g_split_buf[dev]) + 8;  // SplitSync::err (split_sync's layout)
  int v = 0;
  if (hipDeviceSynchronize() != hipSuccess || hipMemcpy(&v, err, sizeof(int), hipMemcpyDeviceToHost) != hipSuccess)
    return 1;
  if (reset && v) {
    const int z = 0;
    (void)hipMemcpy(err, &z, sizeof(int), hipMemcpyHostToDevice);
  }
  return v;
}

bool launch_lstm_seq_fwd(const LstmSeqArgs& a, hipStream_t s) {
  // register-resident K slice: instantiated for the MNIST row-LSTM (I = 28, H = 128)
  if (a.H != 128 || a.I != 28 || a.B % LR || LR * a.I > 1024) return false;
  if (const int ns = split_ns(a)) {
    const SplitSync y = split_sync(s, a.H);
    if (y.llf) {
      auto go = [&](auto nsc) {
        constexpr int NS = decltype(nsc)::value, SPT = split_threads<NS>();
        const size_t lds = ((size_t)LR * (a.I + a.H + 1) + (size_t)LR * (4 * (a.H / NS) + 4)) * sizeof(float);
        auto k = lstm_split_fwd_kernel<128, (28 + 128) / 4, NS>;
        (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (!co_resident((const void*)k, SPT, lds, a.B / LR * NS)) return false;
        hipLaunchKernelGGL(k, dim3(a.B / LR * NS), dim3(SPT), lds, s, a, y);
        return true;
      };
      if (ns == 8 ? go(std::integral_constant<int, 8>{}) : go(std::integral_constant<int, 4>{})) return true;
    }
  }
  LstmSeqArgs b = a;
  if (b.st.x) {  // the single-workgroup-per-group kernel reads xh: stage it first
    launch_seq_stage(b.st, s);
    b.st = SeqStageArgs{};
  }
  const size_t lds = ((size_t)LR * (a.I + a.H + 1) + (size_t)LR * (4 * a.H + 4)) * sizeof(float);
  auto k = lstm_seq_fwd_kernel<128, (28 + 128) / 4>;
  (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(k, dim3(a.B / LR), dim3(1024), lds, s, b);
  return true;
}

bool launch_lstm_seq_bwd(const LstmSeqArgs& a, hipStream_t s) {
  if (a.H != 128 || a.B % LR || (a.I + a.H) % 4) return false;
  if (const int ns = split_ns(a)) {
    const SplitSync y = split_sync(s, a.H);
    if (y.llf) {
      auto go = [&](auto nsc) {
        constexpr int NS = decltype(nsc)::value, SPT = split_threads<NS>();
        const size_t lds = (size_t)2 * 16 * (4 * (a.H / NS) + 4) * sizeof(float);
        auto k = lstm_split_bwd_kernel<128, NS>;
        (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (!co_resident((const void*)k, SPT, lds, a.B / LR * NS)) return false;
        hipLaunchKernelGGL(k, dim3(a.B / LR * NS), dim3(SPT), lds, s, a, y);
        return true;
      };
      if (ns == 8 ? go(std::integral_constant<int, 8>{}) : go(std::integral_constant<int, 4>{})) return true;
    }
  }
  const size_t lds = ((size_t)LR * (4 * a.H + 4) + 2 * (size_t)LR * a.H) * sizeof(float);
  auto k = lstm_seq_bwd_kernel<128>;
  (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(k, dim3(a.B / LR), dim3(1024), lds, s, a);
  return true;
}

}  // namespace dtfe
