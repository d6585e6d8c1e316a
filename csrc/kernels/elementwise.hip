// Memory-bound helper kernels: batch gather from HBM-resident data, noise,
// casts, the small losses of the reference models and bias/activation passes.
// All vectorised where the data layout allows (CDNA guide G13).
#include "elementwise.h"

#include <algorithm>

namespace dtfe {

// last-workgroup counter advance (see optim.hip): every workgroup has read
// *counter before it arrives, so the bump is invisible to this launch.
// Every workgroup read *counter at its start (and used the value, so the load has completed);
// after a barrier one lane takes a ticket and the last one advances the counter.  No data is
// handed between workgroups, so relaxed agent-scope atomics suffice (no fences: a
// __threadfence() costs microseconds per workgroup); the next kernel sees the new value.
__device__ __forceinline__ void advance_counter_last_block(int64_t* counter, uint32_t* done, int64_t by) {
  if (!counter || !done) return;
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t prev = __hip_atomic_fetch_add(done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (prev == gridDim.x * gridDim.y - 1) {
      __hip_atomic_fetch_add((unsigned long long*)counter, (unsigned long long)by, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// 8 source elements -> floats (vector loads: u8 8 B, bf16 16 B, f32 2x16 B)
__device__ __forceinline__ void load8(const void* src, int dt, long off, float (&v)[8]) {
  if (dt == 0) {
    const u32x2_t w = *reinterpret_cast<const u32x2_t*>(reinterpret_cast<const uint8_t*>(src) + off);
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = (float)((w[i >> 2] >> (8 * (i & 3))) & 0xffu) * (1.f / 255.f);
  } else if (dt == 1) {
    const f32x4_t* p = reinterpret_cast<const f32x4_t*>(reinterpret_cast<const float*>(src) + off);
    const f32x4_t lo = p[0], hi = p[1];
#pragma unroll
    for (int i = 0; i < 4; ++i) { v[i] = lo[i]; v[4 + i] = hi[i]; }
  } else {
    const u32x4_t w = *reinterpret_cast<const u32x4_t*>(reinterpret_cast<const bf16*>(src) + off);
    const bf16* e = reinterpret_cast<const bf16*>(&w);
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = bf2f(e[i]);
  }
}

__device__ __forceinline__ long gather_src_row(const GatherArgs& a, int b, int64_t step) {
  if (a.idx) return a.idx[b];
  return (long)(hash_u32(a.seed, (uint64_t)step * a.B + b) % (uint32_t)a.n_rows);
}

// D % 8 == 0: the batch is flattened into 8-element items (row b, chunk d) spread over the whole
// grid, so a few long rows (224x224x3 images) still fill every CU; otherwise one wave per row.
__global__ __launch_bounds__(256) void gather_rows_kernel(GatherArgs a) {
  const int64_t step = a.counter ? *a.counter : 0;
  if ((a.D % 8) == 0) {
    const int cpr = a.D / 8;
    const long n = (long)a.B * cpr;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
      const int b = (int)(i / cpr);
      const int d = (int)(i - (long)b * cpr) * 8;
      const long r = gather_src_row(a, b, step);
      if (a.labels_dst && d == 0) a.labels_dst[b] = a.labels_src[r];
      float v[8];
      load8(a.src, a.src_dtype, r * a.D + d, v);
      const long o = (long)b * a.D + d;
      if (a.dst_dtype == 1) {
        f32x4_t* q = reinterpret_cast<f32x4_t*>(reinterpret_cast<float*>(a.dst) + o);
        q[0] = f32x4_t{v[0], v[1], v[2], v[3]};
        q[1] = f32x4_t{v[4], v[5], v[6], v[7]};
      } else {
        *reinterpret_cast<u32x4_t*>(reinterpret_cast<bf16*>(a.dst) + o) =
            u32x4_t{pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]), pack_bf16x2(v[4], v[5]),
                    pack_bf16x2(v[6], v[7])};
      }
    }
  } else {
    const int lane = threadIdx.x & 63;
    for (int b = blockIdx.x * 4 + (threadIdx.x >> 6); b < a.B; b += gridDim.x * 4) {
      const long r = gather_src_row(a, b, step);
      if (a.labels_dst && lane == 0) a.labels_dst[b] = a.labels_src[r];
      for (int d = lane; d < a.D; d += 64) {
        float v;
        if (a.src_dtype == 0) v = reinterpret_cast<const uint8_t*>(a.src)[r * a.D + d] * (1.f / 255.f);
        else if (a.src_dtype == 1) v = reinterpret_cast<const float*>(a.src)[r * a.D + d];
        else v = bf2f(reinterpret_cast<const bf16*>(a.src)[r * a.D + d]);
        if (a.dst_dtype == 1) reinterpret_cast<float*>(a.dst)[(long)b * a.D + d] = v;
        else reinterpret_cast<bf16*>(a.dst)[(long)b * a.D + d] = f2bf(v);
      }
    }
  }
  if (a.onehot) {
    const long n = (long)a.B * a.ncls;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
      const int b = (int)(i / a.ncls);
      const int c = (int)(i - (long)b * a.ncls);
      a.onehot[i] = a.labels_src[gather_src_row(a, b, step)] == c ? 1.f : 0.f;
    }
  }
  for (int z = 0; z < a.nz; ++z)
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < a.zlen[z]; i += (long)gridDim.x * 256) a.zptr[z][i] = 0u;
  advance_counter_last_block(a.counter, a.done, 1);
}

void launch_gather_rows(const GatherArgs& a, hipStream_t s) {
  long blocks = (a.D % 8) == 0 ? ((long)a.B * (a.D / 8) + 255) / 256 : (a.B + 3) / 4;
  if (blocks > 2048) blocks = 2048;  // (its tail of counter tickets overlaps the grid's drain)
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(gather_rows_kernel, dim3(blocks), dim3(256), 0, s, a);
}

// Optionally also copies ncopy floats (16-B aligned, ncopy % 4 == 0) from csrc to cdst in the same
// launch: the GAN's batch staging (real images into the stacked [real; fake] buffer + the noise).
__global__ __launch_bounds__(256) void uniform_fill_kernel(float* out, long n, float lo, float hi, uint64_t seed,
                                                          int64_t* counter, uint32_t* done, const float* csrc,
                                                          float* cdst, long ncopy) {
  const int64_t step = counter ? *counter : 0;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256)
    out[i] = lo + (hi - lo) * hash_uniform(seed ^ 0xA5A5A5A5ull, (uint64_t)step * n + i);
  for (long i = blockIdx.x * 256L + threadIdx.x; i < ncopy / 4; i += (long)gridDim.x * 256)
    reinterpret_cast<f32x4_t*>(cdst)[i] = reinterpret_cast<const f32x4_t*>(csrc)[i];
  advance_counter_last_block(counter, done, 1);
}

void launch_uniform_fill(float* out, long n, float lo, float hi, uint64_t seed, int64_t* counter, uint32_t* done,
                         hipStream_t s, const float* csrc, float* cdst, long ncopy) {
  const long work = n > ncopy / 4 ? n : ncopy / 4;
  long blocks = (work + 255) / 256;
  if (blocks > (done ? 256 : 1024)) blocks = done ? 256 : 1024;  // see launch_gather_rows
  hipLaunchKernelGGL(uniform_fill_kernel, dim3(blocks), dim3(256), 0, s, out, n, lo, hi, seed, counter, done, csrc,
                     cdst, ncopy);
}

__global__ __launch_bounds__(256) void seq_stage_kernel(SeqStageArgs a) {
  const long tid = blockIdx.x * 256L + threadIdx.x, nth = (long)gridDim.x * 256;
  // x part: one (t, b) row of I floats per I consecutive work items (coalesced reads of image b's
  // row t, coalesced writes of xh row (t, b))
  const long nx = (long)a.T * a.B * a.I;
  for (long i = tid; i < nx; i += nth) {
    const long row = i / a.I, c = i - row * a.I;  // row = t * B + b
    const long t = row / a.B, b = row - t * a.B;
    a.xh[row * a.ld + c] = a.x[(b * a.T + t) * a.I + c];
  }
  const int hw = a.ld - a.I;  // h_{-1} = 0 (step 0 only; later steps are written by the recurrence)
  for (long i = tid; i < (long)a.B * hw; i += nth) {
    const long b = i / hw;
    a.xh[b * a.ld + a.I + (i - b * hw)] = 0.f;
  }
  for (long i = tid; i < a.ny; i += nth) a.ydst[i] = a.ysrc[i];
  for (int z = 0; z < a.nz; ++z)
    for (long i = tid; i < a.zlen[z]; i += nth) a.zptr[z][i] = 0u;
}

void launch_seq_stage(const SeqStageArgs& a, hipStream_t s) {
  long work = (long)a.T * a.B * a.I;
  long blocks = (work + 255) / 256;
  if (blocks > 1024) blocks = 1024;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(seq_stage_kernel, dim3(blocks), dim3(256), 0, s, a);
}

__global__ void cast_f32_bf16_kernel(const float* src, bf16* dst, long n) {
  const long n4 = n / 4;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
    const f32x4_t v = reinterpret_cast<const f32x4_t*>(src)[i];
    u32x2_t o = {pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3])};
    reinterpret_cast<u32x2_t*>(dst)[i] = o;
  }
  for (long i = n4 * 4 + blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) dst[i] = f2bf(src[i]);
}
void launch_cast_f32_bf16(const float* src, bf16* dst, long n, hipStream_t s) {
  long blocks = (n / 4 + 255) / 256 + 1;
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL(cast_f32_bf16_kernel, dim3(blocks), dim3(256), 0, s, src, dst, n);
}
__global__ void cast_bf16_f32_kernel(const bf16* src, float* dst, long n) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) dst[i] = bf2f(src[i]);
}
void launch_cast_bf16_f32(const bf16* src, float* dst, long n, hipStream_t s) {
  long blocks = (n + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL(cast_bf16_f32_kernel, dim3(blocks), dim3(256), 0, s, src, dst, n);
}

// one wave per row
__global__ __launch_bounds__(256) void softmax_xent_kernel(XentArgs a) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= a.B) return;
  const float* lg = a.logits + (long)row * a.NC;
  float mx = -INFINITY;
  int am = 0;
  for (int n = lane; n < a.NC; n += 64) if (lg[n] > mx) { mx = lg[n]; am = n; }
  // wave argmax (first max)
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float om = __shfl_xor(mx, o, 64);
    const int oa = __shfl_xor(am, o, 64);
    if (om > mx || (om == mx && oa < am)) { mx = om; am = oa; }
  }
  float se = 0.f;
  for (int n = lane; n < a.NC; n += 64) se += __expf(lg[n] - mx);
  se = wave_sum(se);
  const float lse = mx + __logf(se);
  float loss = 0.f;
  int label = -1;
  if (a.labels_i) label = a.labels_i[row];
  float ymax = -1.f;
  int yarg = 0;
  for (int n = lane; n < a.NC; n += 64) {
    const float y = a.labels_i ? (n == label ? 1.f : 0.f) : a.labels_oh[(long)row * a.NC + n];
    const float p = __expf(lg[n] - lse);
    loss += y * (lse - lg[n]);
    if (a.dlogits) a.dlogits[(long)row * a.NC + n] = (p - y) * a.scale;
    if (a.probs) a.probs[(long)row * a.NC + n] = p;
    if (y > ymax) { ymax = y; yarg = n; }
  }
  loss = wave_sum(loss);
  if (!a.labels_i) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float om = __shfl_xor(ymax, o, 64);
      const int oa = __shfl_xor(yarg, o, 64);
      if (om > ymax || (om == ymax && oa < yarg)) { ymax = om; yarg = oa; }
    }
    label = yarg;
  }
  if (lane == 0) {
    if (a.loss_rows) a.loss_rows[row] = loss;
    if (a.loss_sum) atomicAdd(a.loss_sum, loss);
    if (a.correct) atomicAdd(a.correct, (int)(am == label));
  }
}
void launch_softmax_xent(const XentArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(softmax_xent_kernel, dim3((a.B + 3) / 4), dim3(256), 0, s, a);
}

// F32: fp32 features / feature gradient (the LSTM's fp32 head), else bf16 (ResNet's pooled features);
// WFM: W and dW are [F][NC] (the LSTM's Variable (128, 10)), else [NC][F].
// One 1024-thread workgroup, every phase spread so that no thread runs a long dependent chain (the
// first form - one output per thread, 128-long fmaf chains over LDS - took 20-24 us, latency-bound):
//   logits   thread = (row, class): 16-B reads of the feature and weight rows, four independent
//            fmaf chains (features f = 4i + e), summed pairwise
//   softmax  one thread per row (softmax_xent_kernel's expressions)
//   dW, db   thread = (class c, 4 features, batch slice): 16-B feature reads, 4 independent chains,
//            the slices summed in a fixed order through LDS
//   dfeat    thread = (row, 4 or 8 features): NC fmaf each, one 16-B store
constexpr int DH_NCMAX = 16;
template <bool F32, bool WFM>
__global__ __launch_bounds__(1024) void dense_head_kernel(DenseHeadArgs a) {
  extern __shared__ float hsm[];
  const int B = a.B, F = a.F, NC = a.NC, FP = F + 4, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  float* sf = hsm;             // [B][F+4] features (fp32; 16-B aligned rows)
  float* sw = sf + B * FP;     // [NC][F+4] weights
  float* sd = sw + NC * FP;    // [B][NC] logits, then dlogits
  float* sy = sd + B * NC;     // [B][NC] labels (a.ylds: staged with the features, the softmax rows read LDS)
  float* red = sy + (a.ylds ? B * NC : 0);  // [2][32] block-reduce scratch, then the dW slice partials
  constexpr int EPC = F32 ? 4 : 8;
  const int CPR = F / EPC;
  for (int i = tid; i < ((a.diag & 32) ? 0 : B * CPR); i += 1024) {
    const int b = i / CPR, f0 = (i - b * CPR) * EPC;
    if constexpr (F32) {
      *reinterpret_cast<f32x4_t*>(sf + b * FP + f0) = reinterpret_cast<const f32x4_t*>(a.feat)[i];
    } else {
      const u32x4_t v = reinterpret_cast<const u32x4_t*>(a.feat)[i];
      f32x4_t lo, hi;
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        lo[2 * e] = __uint_as_float(v[e] << 16);
        lo[2 * e + 1] = __uint_as_float(v[e] & 0xffff0000u);
        hi[2 * e] = __uint_as_float(v[2 + e] << 16);
        hi[2 * e + 1] = __uint_as_float(v[2 + e] & 0xffff0000u);
      }
      *reinterpret_cast<f32x4_t*>(sf + b * FP + f0) = lo;
      *reinterpret_cast<f32x4_t*>(sf + b * FP + f0 + 4) = hi;
    }
  }
  for (int i = tid; i < (a.ylds ? B * NC : 0); i += 1024) sy[i] = a.y[i];
  for (int i = tid; i < NC * F; i += 1024) {
    if constexpr (WFM) {
      const int f = i / NC, c = i - f * NC;
      sw[c * FP + f] = a.w[i];
    } else {
      const int c = i / F, f = i - c * F;
      sw[c * FP + f] = a.w[i];
    }
  }
  __syncthreads();
  for (int o = tid; o < ((a.diag & 1) ? 0 : B * NC); o += 1024) {  // logits: 16-B row reads, four independent fmaf chains
    const int b = o / NC, c = o - b * NC;
    f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
    for (int f = 0; f < F; f += 4) {
      const f32x4_t x = *reinterpret_cast<const f32x4_t*>(sf + b * FP + f);
      const f32x4_t w = *reinterpret_cast<const f32x4_t*>(sw + c * FP + f);
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[e] = __builtin_fmaf(x[e], w[e], acc[e]);
    }
    const float v = (acc[0] + acc[1]) + (acc[2] + acc[3]) + (a.bias ? a.bias[c] : 0.f);
    sd[o] = v;
    if (a.logits) a.logits[o] = v;
  }
  __syncthreads();
  // rows: softmax_xent_kernel's expressions (first-max argmax, lse, loss, (p - y) * scale)
  float loss = 0.f, hits = 0.f;
  for (int b = tid; b < ((a.diag & 2) ? 0 : B); b += 1024) {
    float* l = sd + b * NC;
    const float* y = a.ylds ? sy + b * NC : a.y + (long)b * NC;
    float mx = -INFINITY, ymax = -1.f;
    int am = 0, yarg = 0;
    for (int c = 0; c < NC; ++c) {
      if (l[c] > mx) { mx = l[c]; am = c; }
      if (y[c] > ymax) { ymax = y[c]; yarg = c; }
    }
    float se = 0.f;
    for (int c = 0; c < NC; ++c) se += __expf(l[c] - mx);
    const float lse = mx + __logf(se);
    for (int c = 0; c < NC; ++c) {
      const float p = __expf(l[c] - lse);
      loss += y[c] * (lse - l[c]);
      l[c] = (p - y[c]) * a.scale;
    }
    hits += am == yarg ? 1.f : 0.f;
  }
  loss = wave_sum(loss);
  hits = wave_sum(hits);
  if (lane == 0) {
    red[wid] = loss;
    red[32 + wid] = hits;
  }
  __syncthreads();
  if (tid == 0) {
    float tl = 0.f, th = 0.f;
    for (int w = 0; w < 16; ++w) {
      tl += red[w];
      th += red[32 + w];
    }
    if (a.loss_sum) atomicAdd(a.loss_sum, tl);
    if (a.correct) atomicAdd(a.correct, (int)th);
  }
  __syncthreads();  // (red is reused below)
  // dW[c][f..f+3] over a batch slice: items (c, f4) x S slices, S = 1024 / (NC * F / 4) (<= 8)
  const int F4 = F / 4, NI = NC * F4, S = a.slices;
  float* part = red + 64;  // [S][NI][4] (S > 1)
  for (int t = tid; t < ((a.diag & 4) ? 0 : NI * S); t += 1024) {
    const int s = t / NI, it = t - s * NI, c = it / F4, f = (it - c * F4) * 4;
    const int b0 = s * B / S, b1 = (s + 1) * B / S;
    f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
    for (int b = b0; b < b1; ++b) {
      const float d = sd[b * NC + c];
      const f32x4_t x = *reinterpret_cast<const f32x4_t*>(sf + b * FP + f);
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[e] = __builtin_fmaf(d, x[e], acc[e]);
    }
    if (S > 1) {
      *reinterpret_cast<f32x4_t*>(part + ((long)s * NI + it) * 4) = acc;
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const long o = WFM ? (long)(f + e) * NC + c : (long)c * F + f + e;
        a.dw[o] = a.store ? acc[e] : a.dw[o] + acc[e];
      }
    }
  }
  if (wid < NC && a.db && !(a.diag & 16)) {  // db[c]: wave c, rows strided over the lanes + a butterfly
    float acc = 0.f;
    for (int b = lane; b < B; b += 64) acc += sd[b * NC + wid];
    acc = wave_sum(acc);
    if (lane == 0) a.db[wid] = a.store ? acc : a.db[wid] + acc;
  }
  __syncthreads();
  for (int it = tid; it < (S > 1 && !(a.diag & 4) ? NI : 0); it += 1024) {
    f32x4_t g = *reinterpret_cast<const f32x4_t*>(part + (long)it * 4);
    for (int s = 1; s < S; ++s) g += *reinterpret_cast<const f32x4_t*>(part + ((long)s * NI + it) * 4);
    const int c = it / F4, f = (it - c * F4) * 4;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const long o = WFM ? (long)(f + e) * NC + c : (long)c * F + f + e;
      a.dw[o] = a.store ? g[e] : a.dw[o] + g[e];
    }
  }
  if (a.dl_out)
    for (int o = tid; o < B * NC; o += 1024) a.dl_out[o] = sd[o];
  for (int i = tid; i < ((a.diag & 8) || !a.dfeat ? 0 : B * CPR); i += 1024) {  // dfeat = dlogits W, one 16-B store per chunk
    const int b = i / CPR, f0 = (i - b * CPR) * EPC;
    float acc[EPC] = {};
    for (int c = 0; c < NC; ++c) {
      const float dl = sd[b * NC + c];
#pragma unroll
      for (int e = 0; e < EPC; ++e) acc[e] = __builtin_fmaf(dl, sw[c * FP + f0 + e], acc[e]);
    }
    if constexpr (F32) {
      reinterpret_cast<f32x4_t*>(a.dfeat)[i] = f32x4_t{acc[0], acc[1], acc[2], acc[3]};
    } else {
      u32x4_t o;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = pack_bf16x2(acc[2 * e], acc[2 * e + 1]);
      reinterpret_cast<u32x4_t*>(a.dfeat)[i] = o;
    }
  }
}

bool launch_dense_head(const DenseHeadArgs& a, hipStream_t s) {
  // LDS: features + weights [.][F+4], logits [B][NC], 64 reduce floats, dW slice partials (S x NI x 4)
  const long ni = (long)a.NC * (a.F / 4), base0 = ((long)(a.B + a.NC) * (a.F + 4) + (long)a.B * a.NC + 64) * 4;
  const bool ylds = base0 + (long)a.B * a.NC * 4 <= 150 * 1024;
  const long base = base0 + (ylds ? (long)a.B * a.NC * 4 : 0);
  long sl = ni >= 1024 ? 1 : std::min<long>(8, 1024 / ni);
  while (sl > 1 && base + sl * ni * 16 > 150 * 1024) --sl;
  const size_t lds = (size_t)(base + (sl > 1 ? sl * ni * 16 : 0));
  if (lds > 150 * 1024 || a.NC > DH_NCMAX || a.F % 8 || !a.dw || (!a.dfeat && !a.dl_out)) return false;
  DenseHeadArgs ad = a;
  ad.slices = (int)sl;
  ad.ylds = ylds ? 1 : 0;
  ad.diag = diag_bits("dh");
  auto go = [&](auto kern) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(kern, dim3(1), dim3(1024), lds, s, ad);
  };
  if (a.f32) {
    if (a.w_fmajor) go(dense_head_kernel<true, true>);
    else go(dense_head_kernel<true, false>);
  } else {
    if (a.w_fmajor) go(dense_head_kernel<false, true>);
    else go(dense_head_kernel<false, false>);
  }
  return true;
}

__global__ __launch_bounds__(256) void gan_loss_kernel(GanLossArgs a) {
  __shared__ float sg[4], sd[4];
  float gl = 0.f, dl = 0.f;
  const float invB = 1.f / a.B;
  for (int i = threadIdx.x; i < a.B; i += 256) {
    float pr = a.d_real[i], pf = a.d_fake[i];
    float pr_c = pr, pf_c = pf, qf_c = 1.f - pf;
    if (a.clamp_eps > 0.f) {
      pr_c = fmaxf(pr, a.clamp_eps);
      pf_c = fmaxf(pf, a.clamp_eps);
      qf_c = fmaxf(1.f - pf, a.clamp_eps);
    }
    gl += -logf(pf_c);
    dl += -(logf(pr_c) + logf(qf_c));
    // d/dz of -log(sigmoid(z)) = -(1 - s);  d/dz of -log(1 - sigmoid(z)) = s
    a.dz_real_disc[i] = -(1.f - pr) * invB;
    a.dz_fake_disc[i] = pf * invB;
    a.dz_fake_gen[i] = -(1.f - pf) * invB;
  }
  gl = wave_sum(gl);
  dl = wave_sum(dl);
  if ((threadIdx.x & 63) == 0) { sg[threadIdx.x >> 6] = gl; sd[threadIdx.x >> 6] = dl; }
  __syncthreads();
  if (threadIdx.x == 0) {
    *a.gen_loss = (sg[0] + sg[1] + sg[2] + sg[3]) * invB;
    *a.disc_loss = (sd[0] + sd[1] + sd[2] + sd[3]) * invB;
  }
}
void launch_gan_loss(const GanLossArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(gan_loss_kernel, dim3(1), dim3(256), 0, s, a);
}

// ws == nullptr: one float atomic per workgroup into a loss the launcher zeroed (a memset node).  With ws
// (MSE_WS_FLOATS, zero-initialised): each workgroup leaves its partial in a write-through store and takes a
// ticket (the split-K hand-off of gemm_dense.h); the last arriver sums the partials in workgroup order and
// STORES the loss - one launch, no memset, a bitwise-reproducible loss.
template <bool TICKET>
__global__ __launch_bounds__(256) void mse_sigmoid_kernel(const float* y, const float* t, long n, float* loss,
                                                          float* dz, float* ws) {
  __shared__ float part[4];
  float acc = 0.f;
  const float inv = 1.f / (float)n;
  const long n4 = n / 4, nth = (long)gridDim.x * 256, tid = blockIdx.x * 256L + threadIdx.x;
  for (long i = tid; i < n4; i += nth) {  // torch allocations: 16-B aligned
    const f32x4_t yv = reinterpret_cast<const f32x4_t*>(y)[i], tv = reinterpret_cast<const f32x4_t*>(t)[i];
    f32x4_t o;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float d = yv[e] - tv[e];
      acc += d * d;
      o[e] = 2.f * d * inv * yv[e] * (1.f - yv[e]);
    }
    reinterpret_cast<f32x4_t*>(dz)[i] = o;
  }
  for (long i = 4 * n4 + tid; i < n; i += nth) {
    const float d = y[i] - t[i];
    acc += d * d;
    dz[i] = 2.f * d * inv * y[i] * (1.f - y[i]);
  }
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = acc;
  __syncthreads();
  const float v = ((part[0] + part[1]) + part[2]) + part[3];
  if constexpr (!TICKET) {
    if (threadIdx.x == 0) atomicAdd(loss, v * inv);
  } else {
    __shared__ int lastf;
    __shared__ float part2[4];
    if (threadIdx.x == 0) {
      const __amdgpu_buffer_rsrc_t slot = __builtin_amdgcn_make_buffer_rsrc(ws, (short)0, MSE_PARTS * 4, 0x00020000);
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), slot, blockIdx.x * 4, 0, 16);  // write-through
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      int* ctr = reinterpret_cast<int*>(ws + MSE_PARTS);
      const int prev = __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = prev == (int)gridDim.x - 1;
      if (last) {
        __hip_atomic_store(ctr, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // next launch / replay
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      lastf = last;
    }
    __syncthreads();
    if (!lastf) return;
    // the last arriver: one partial per thread (<= MSE_PARTS), a fixed butterfly + wave order
    float x = (int)threadIdx.x < (int)gridDim.x ? ws[threadIdx.x] : 0.f;
    x = wave_sum(x);
    if ((threadIdx.x & 63) == 0) part2[threadIdx.x >> 6] = x;
    __syncthreads();
    if (threadIdx.x == 0) *loss = (((part2[0] + part2[1]) + part2[2]) + part2[3]) * inv;
  }
}
void launch_mse_sigmoid(const float* y, const float* t, long n, float* loss, float* dz, hipStream_t s, float* ws) {
  long blocks = (n / 4 + 255) / 256;
  if (blocks > (ws ? MSE_PARTS : 512)) blocks = ws ? MSE_PARTS : 512;
  if (blocks < 1) blocks = 1;
  if (ws) {
    hipLaunchKernelGGL(mse_sigmoid_kernel<true>, dim3(blocks), dim3(256), 0, s, y, t, n, loss, dz, ws);
    return;
  }
  hipMemsetAsync(loss, 0, sizeof(float), s);
  hipLaunchKernelGGL(mse_sigmoid_kernel<false>, dim3(blocks), dim3(256), 0, s, y, t, n, loss, dz, ws);
}

// column sums: block = 64 columns x 4 row-groups
__global__ __launch_bounds__(256) void colsum_kernel(const void* x, int x_f32, int M, int N, long ld, float* db,
                                                     float scale) {
  __shared__ float part[4][64];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int rg = threadIdx.x >> 6;
  float acc = 0.f;
  if (c < N) {
    for (int m = blockIdx.y * 4 + rg; m < M; m += gridDim.y * 4) {
      acc += x_f32 ? reinterpret_cast<const float*>(x)[(long)m * ld + c]
                   : bf2f(reinterpret_cast<const bf16*>(x)[(long)m * ld + c]);
    }
  }
  part[rg][threadIdx.x & 63] = acc;
  __syncthreads();
  if (rg == 0 && c < N) {
    const float s = part[0][threadIdx.x] + part[1][threadIdx.x] + part[2][threadIdx.x] + part[3][threadIdx.x];
    atomicAdd(db + c, s * scale);
  }
}
void launch_colsum(const void* x, int x_f32, int M, int N, long ld, float* db, float scale, hipStream_t s) {
  // enough row groups that each thread sums only a few rows (the sums are latency-bound
  // dependent chains otherwise) while the grid still fills the CUs
  int gx = (N + 63) / 64;
  int gy = (M + 31) / 32;
  if (gy * gx > 1024) gy = (1024 + gx - 1) / gx;
  if (gy < 1) gy = 1;
  hipLaunchKernelGGL(colsum_kernel, dim3(gx, gy), dim3(256), 0, s, x, x_f32, M, N, ld, db, scale);
}

__global__ void act_grad_kernel(const float* dy, const float* y, float* dz, long n, int act) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256)
    dz[i] = dy[i] * act_grad_from_out(y[i], act);
}
void launch_act_grad(const float* dy, const float* y, float* dz, long n, int act, hipStream_t s) {
  long blocks = (n + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL(act_grad_kernel, dim3(blocks), dim3(256), 0, s, dy, y, dz, n, act);
}

__global__ void bias_act_kernel(BiasActArgs a) {
  const long n = (long)a.M * a.N;
  const int64_t step = a.counter ? *a.counter : 0;
  const float inv_keep = 1.f / a.keep;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    float v = a.x[i] + (a.bias ? a.bias[i % a.N] : 0.f);
    v = apply_act(v, a.act);
    if (a.keep < 1.f) v = hash_uniform(a.seed, (uint64_t)step * n + i) < a.keep ? v * inv_keep : 0.f;
    if (a.out_f32) reinterpret_cast<float*>(a.out)[i] = v;
    else reinterpret_cast<bf16*>(a.out)[i] = f2bf(v);
  }
}
__global__ void lstm_cell_fwd_kernel(LstmCellArgs a) {
  const long n = (long)a.B * a.H;
  for (long idx = blockIdx.x * 256L + threadIdx.x; idx < n; idx += (long)gridDim.x * 256) {
    const long b = idx / a.H;
    const int u = (int)(idx % a.H);
    const float* g = a.gates + b * 4 * a.H;
    const float si = sigmoidf_(g[u]);
    const float tj = tanhf(g[a.H + u]);
    const float sf = sigmoidf_(g[2 * a.H + u] + a.forget_bias);
    const float so = sigmoidf_(g[3 * a.H + u]);
    const float cp = a.c_prev ? a.c_prev[idx] : 0.f;
    const float c = cp * sf + si * tj;
    a.c[idx] = c;
    a.h_out[b * a.ld_h + u] = tanhf(c) * so;
    float* ac = a.act + b * 4 * a.H;
    ac[u] = si;
    ac[a.H + u] = tj;
    ac[2 * a.H + u] = sf;
    ac[3 * a.H + u] = so;
  }
}
void launch_lstm_cell_fwd(const LstmCellArgs& a, hipStream_t s) {
  long blocks = ((long)a.B * a.H + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL(lstm_cell_fwd_kernel, dim3(blocks), dim3(256), 0, s, a);
}

__global__ void lstm_cell_bwd_kernel(LstmCellArgs a) {
  const long n = (long)a.B * a.H;
  for (long idx = blockIdx.x * 256L + threadIdx.x; idx < n; idx += (long)gridDim.x * 256) {
    const long b = idx / a.H;
    const int u = (int)(idx % a.H);
    const float* ac = a.act + b * 4 * a.H;
    const float si = ac[u], tj = ac[a.H + u], sf = ac[2 * a.H + u], so = ac[3 * a.H + u];
    const float c = a.c[idx];
    const float cp = a.c_prev ? a.c_prev[idx] : 0.f;
    float dh = a.dh ? a.dh[idx] : 0.f;
    if (a.dh2) dh += a.dh2[idx];
    const float tc = tanhf(c);
    const float dc = (a.dc_next ? a.dc_next[idx] : 0.f) + dh * so * (1.f - tc * tc);
    float* dg = a.dgates + b * 4 * a.H;
    dg[u] = dc * tj * si * (1.f - si);
    dg[a.H + u] = dc * si * (1.f - tj * tj);
    dg[2 * a.H + u] = dc * cp * sf * (1.f - sf);
    dg[3 * a.H + u] = dh * tc * so * (1.f - so);
    a.dc_prev[idx] = dc * sf;
  }
}
void launch_lstm_cell_bwd(const LstmCellArgs& a, hipStream_t s) {
  long blocks = ((long)a.B * a.H + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL(lstm_cell_bwd_kernel, dim3(blocks), dim3(256), 0, s, a);
}

void launch_bias_act(const BiasActArgs& a, hipStream_t s) {
  long n = (long)a.M * a.N;
  long blocks = (n + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL(bias_act_kernel, dim3(blocks), dim3(256), 0, s, a);
}

}  // namespace dtfe
