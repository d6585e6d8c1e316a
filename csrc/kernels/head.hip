// Fused classifier head, per-row part (MNIST CNN: fc 1024 -> 10):
//
//   logits = h . W^T + b                    (h: post-ReLU/dropout activations, bf16)
//   loss   = sum softmax_cross_entropy(logits, labels)          (atomic scalar)
//   dlogit = (softmax - onehot) * scale                         (bf16 [B][ld_dl])
//   dZ     = (dlogit . W) * inv_keep * (h > 0)                  (bf16 [B][K])
//
// One wave per batch row (K/64 features per lane, W resident in LDS as f32);
// the 10 logits are 10 wave reductions and the softmax runs on wave-uniform
// registers.  The weight/bias gradients of this layer (dW = dlogit^T h,
// db = sum dlogit) are a separate split-K MFMA GEMM reading the bf16 dlogit
// rows this kernel writes; the bias gradient of the layer below comes out of
// that layer's wgrad GEMM through its ones column.  Replaces TF's MatMul +
// BiasAdd + SoftmaxCrossEntropyWithLogits + MatMul-grad + ReluGrad chain
// (SURVEY K01/K02/K07).
#include "common.h"
#include "head.h"

namespace dtfe {

// One wave per batch row (K/64 features per lane).  The wave's slice of W (NC x K/64 bf16,
// 80 VGPRs for 10 x 16) is loaded straight into registers together with the h row - one
// round of global loads, no LDS staging and no barrier (the earlier LDS-staged version spent
// most of its ~20 us in the serial W staging of every workgroup); the NC dot products are
// reduced across the wave with independent butterfly chains that the scheduler interleaves.
template <int NC, int K>
__global__ __launch_bounds__(256) void head_xent_kernel(HeadArgs a) {
  constexpr int E = K / 64;  // features per lane
  static_assert(E % 8 == 0, "K must be a multiple of 512");
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  __shared__ float red_loss[4];
  __shared__ int red_correct[4];
  if (a.step_counter && blockIdx.x == 0 && threadIdx.x == 0) *a.step_counter += 1;
  const int row = min(blockIdx.x * 4 + wid, a.B - 1);  // a surplus wave recomputes the last row, unstored
  const bool live = blockIdx.x * 4 + wid < a.B;
  u32x4_t wv[NC][E / 8], hv[E / 8];
#pragma unroll
  for (int c = 0; c < E / 8; ++c) hv[c] = *reinterpret_cast<const u32x4_t*>(a.h + (long)row * K + lane * E + c * 8);
#pragma unroll
  for (int n = 0; n < NC; ++n)
#pragma unroll
    for (int c = 0; c < E / 8; ++c) wv[n][c] = *reinterpret_cast<const u32x4_t*>(a.w + (long)n * K + lane * E + c * 8);
  const int label = a.labels[row];
  float bias[NC];
#pragma unroll
  for (int n = 0; n < NC; ++n) bias[n] = a.b ? a.b[n] : 0.f;

  float h[E];
#pragma unroll
  for (int c = 0; c < E / 8; ++c)
#pragma unroll
    for (int i = 0; i < 8; ++i) h[c * 8 + i] = bf2f((bf16)(hv[c][i >> 1] >> (16 * (i & 1))));
  auto wel = [&](int n, int i) { return bf2f((bf16)(wv[n][i / 8][(i % 8) >> 1] >> (16 * (i & 1)))); };
  float logit[NC];
#pragma unroll
  for (int n = 0; n < NC; ++n) {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < E; ++i) s = fmaf(h[i], wel(n, i), s);
    logit[n] = s;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1)
#pragma unroll
    for (int n = 0; n < NC; ++n) logit[n] += __shfl_xor(logit[n], o, 64);
#pragma unroll
  for (int n = 0; n < NC; ++n) logit[n] += bias[n];

  float mx = logit[0];
  int am = 0;
#pragma unroll
  for (int n = 1; n < NC; ++n) if (logit[n] > mx) { mx = logit[n]; am = n; }
  float se = 0.f;
#pragma unroll
  for (int n = 0; n < NC; ++n) se += __expf(logit[n] - mx);
  const float lse = mx + __logf(se);
  float dl[NC];
  float lg_label = 0.f;
#pragma unroll
  for (int n = 0; n < NC; ++n) {
    const float p = __expf(logit[n] - lse);
    dl[n] = (p - (n == label ? 1.f : 0.f)) * a.scale;
    if (n == label) lg_label = logit[n];
  }
  if (live && lane < a.ld_dl) {
    float v = 0.f, lv = 0.f;
#pragma unroll
    for (int n = 0; n < NC; ++n) if (n == lane) { v = dl[n]; lv = logit[n]; }
    a.dl[(long)row * a.ld_dl + lane] = f2bf(v);  // pad columns get 0
    if (a.logits_out && lane < NC) a.logits_out[(long)row * NC + lane] = lv;
  }
  u32x4_t outv[E / 8];
#pragma unroll
  for (int i = 0; i < E; ++i) {
    float g = 0.f;
#pragma unroll
    for (int n = 0; n < NC; ++n) g = fmaf(dl[n], wel(n, i), g);
    g = h[i] > 0.f ? g * a.inv_keep : 0.f;
    reinterpret_cast<bf16*>(&outv[i / 8])[i % 8] = f2bf(g);
  }
  if (live)
#pragma unroll
    for (int c = 0; c < E / 8; ++c) *reinterpret_cast<u32x4_t*>(a.dz + (long)row * K + lane * E + c * 8) = outv[c];
  // one atomic per workgroup (1024 same-address atomics per launch would serialise)
  if (lane == 0) {
    red_loss[wid] = live ? lse - lg_label : 0.f;
    red_correct[wid] = live && am == label;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    if (a.loss_sum) atomicAdd(a.loss_sum, red_loss[0] + red_loss[1] + red_loss[2] + red_loss[3]);
    if (a.correct) atomicAdd(a.correct, red_correct[0] + red_correct[1] + red_correct[2] + red_correct[3]);
  }
}

void launch_head_xent(const HeadArgs& a, hipStream_t s) {
  if (a.NC != 10 || a.K != 1024) throw std::runtime_error("head_xent: only NC=10, K=1024 instantiated");
  const int blocks = (a.B + 3) / 4;  // one row per wave
  hipLaunchKernelGGL((head_xent_kernel<10, 1024>), dim3(blocks), dim3(256), 0, s, a);
}

}  // namespace dtfe

namespace dtfe {

// Classifier-head weight / bias gradient: dW[c][k] = sum_b dl[b][c] h[b][k], db[c] = sum_b dl[b][c].
// The layer is 10 x 1024 over a 1024-row batch (21 MFLOP): a split-K MFMA GEMM spends ~16 us on
// 32 x 32 tiles (a 10-row M padded to 32) and the fixed-order combine of 8 K-splits.  Here one
// 1024-thread workgroup owns 16 columns of dW for the WHOLE batch (no cross-workgroup
// reduction): the batch's dlogit rows are staged in LDS (32 KB, 16-B loads) while every thread
// has its 16 h values in flight (thread (column c = t & 15, row group r = t >> 4) takes rows
// r, r + 64, ...), so the launch pays about two memory latencies; the 64 row groups are then
// summed through LDS in a fixed order - bitwise reproducible, no atomics.  Workgroup K/16
// produces the bias gradient (h read as ones).
template <int NC>
__global__ __launch_bounds__(1024) void head_wgrad_kernel(HeadWgradArgs a) {
  constexpr int RG = 64, PER = 16;  // row groups, rows per thread (B <= RG * PER)
  // one LDS buffer: the staged dlogit rows, then (after a barrier) the per-row-group partials
  constexpr int DL_BYTES = RG * PER * 16 * 2, PART_BYTES = RG * 16 * (NC + 1) * 4;
  __shared__ __attribute__((aligned(16))) char smem[DL_BYTES > PART_BYTES ? DL_BYTES : PART_BYTES];
  auto dls = reinterpret_cast<bf16(*)[16]>(smem);
  auto part = reinterpret_cast<float(*)[16][NC + 1]>(smem);
  const int t = threadIdx.x, c = t & 15, rg = t >> 4;
  const bool bias_blk = blockIdx.x * 16 >= a.K;
  const int col = blockIdx.x * 16 + c;
  float hv[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int b = rg + RG * i;
    hv[i] = b < a.B ? (bias_blk ? 1.f : bf2f(a.h[(long)b * a.ldh + col])) : 0.f;
  }
  for (int i = t; i < RG * PER * 2; i += 1024) {  // 16-B halves of the 32-B dlogit rows
    const int b = i >> 1;
    u32x4_t v = {0u, 0u, 0u, 0u};
    if (b < a.B) v = *reinterpret_cast<const u32x4_t*>(a.dl + (long)b * a.ld_dl + (i & 1) * 8);
    *reinterpret_cast<u32x4_t*>(&dls[b][(i & 1) * 8]) = v;
  }
  __syncthreads();
  float acc[NC];
#pragma unroll
  for (int n = 0; n < NC; ++n) acc[n] = 0.f;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int b = rg + RG * i;
    const u32x4_t d0 = *reinterpret_cast<const u32x4_t*>(&dls[b][0]);
    const u32x4_t d1 = *reinterpret_cast<const u32x4_t*>(&dls[b][8]);
#pragma unroll
    for (int n = 0; n < NC; ++n) {
      const uint32_t w = n < 8 ? d0[n >> 1] : d1[(n - 8) >> 1];
      acc[n] = fmaf(bf2f((bf16)(w >> (16 * (n & 1)))), hv[i], acc[n]);
    }
  }
  __syncthreads();  // every thread is done with the staged rows
#pragma unroll
  for (int n = 0; n < NC; ++n) part[rg][c][n] = acc[n];
  __syncthreads();
  if (t < 16 * NC) {
    const int cc = t % 16, n = t / 16;
    float s = 0.f;
    for (int r = 0; r < RG; ++r) s += part[r][cc][n];
    if (!bias_blk) a.dw[(long)n * a.ldw + blockIdx.x * 16 + cc] = s * a.scale;
    else if (cc == 0) a.db[n] = s * a.scale;
  }
}

void launch_head_wgrad(const HeadWgradArgs& a, hipStream_t s) {
  if (a.NC != 10 || a.K % 16 || a.ld_dl < 16 || a.ld_dl % 8 || a.B > 1024)
    throw std::runtime_error("head_wgrad: needs NC=10, K % 16 == 0, 16-B aligned dl rows of >= 16, B <= 1024");
  const int blocks = a.K / 16 + (a.db ? 1 : 0);
  hipLaunchKernelGGL(head_wgrad_kernel<10>, dim3(blocks), dim3(1024), 0, s, a);
}

}  // namespace dtfe
