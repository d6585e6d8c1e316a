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

template <int NC, int K>
__global__ __launch_bounds__(256) void head_xent_kernel(HeadArgs a) {
  constexpr int E = K / 64;  // features per lane
  static_assert(E % 8 == 0, "K must be a multiple of 512");
  __shared__ __attribute__((aligned(16))) float wl[NC * K];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (int i = threadIdx.x * 8; i < NC * K; i += 256 * 8) {
    const u32x4_t v = *reinterpret_cast<const u32x4_t*>(a.w + i);
    const bf16* e = reinterpret_cast<const bf16*>(&v);
#pragma unroll
    for (int j = 0; j < 8; ++j) wl[i + j] = bf2f(e[j]);
  }
  float bias[NC];
#pragma unroll
  for (int n = 0; n < NC; ++n) bias[n] = a.b ? a.b[n] : 0.f;
  __syncthreads();

  float loss_acc = 0.f;
  int correct = 0;
  const int waves_total = gridDim.x * 4;
  for (int row = blockIdx.x * 4 + wid; row < a.B; row += waves_total) {
    float h[E];
#pragma unroll
    for (int c = 0; c < E / 8; ++c) {
      const u32x4_t v = *reinterpret_cast<const u32x4_t*>(a.h + (long)row * K + lane * E + c * 8);
      const bf16* e = reinterpret_cast<const bf16*>(&v);
#pragma unroll
      for (int i = 0; i < 8; ++i) h[c * 8 + i] = bf2f(e[i]);
    }
    float logit[NC];
#pragma unroll
    for (int n = 0; n < NC; ++n) {
      const f32x4_t* wr = reinterpret_cast<const f32x4_t*>(wl + n * K + lane * E);
      float s = 0.f;
#pragma unroll
      for (int i = 0; i < E / 4; ++i) {
        const f32x4_t w4 = wr[i];
        s = fmaf(h[4 * i], w4[0], s);
        s = fmaf(h[4 * i + 1], w4[1], s);
        s = fmaf(h[4 * i + 2], w4[2], s);
        s = fmaf(h[4 * i + 3], w4[3], s);
      }
      logit[n] = wave_sum(s) + bias[n];
    }
    const int label = a.labels[row];
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
    loss_acc += lse - lg_label;
    correct += (am == label);
    if (lane < a.ld_dl) {
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
      for (int n = 0; n < NC; ++n) g = fmaf(dl[n], wl[n * K + lane * E + i], g);
      g = h[i] > 0.f ? g * a.inv_keep : 0.f;
      reinterpret_cast<bf16*>(&outv[i / 8])[i % 8] = f2bf(g);
    }
#pragma unroll
    for (int c = 0; c < E / 8; ++c)
      *reinterpret_cast<u32x4_t*>(a.dz + (long)row * K + lane * E + c * 8) = outv[c];
  }
  if (lane == 0) {
    if (a.loss_sum) atomicAdd(a.loss_sum, loss_acc);
    if (a.correct) atomicAdd(a.correct, correct);
  }
}

void launch_head_xent(const HeadArgs& a, hipStream_t s) {
  if (a.NC != 10 || a.K != 1024) throw std::runtime_error("head_xent: only NC=10, K=1024 instantiated");
  int blocks = (a.B + 3) / 4;  // one row per wave
  if (blocks > 1024) blocks = 1024;
  hipLaunchKernelGGL((head_xent_kernel<10, 1024>), dim3(blocks), dim3(256), 0, s, a);
}

}  // namespace dtfe
