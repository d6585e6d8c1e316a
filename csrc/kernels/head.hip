// Fused classifier head for the CNN family (MNIST CNN: fc 1024 -> 10):
//
//   logits = h . W^T + b                    (h: post-ReLU/dropout activations, bf16)
//   loss   = mean softmax_cross_entropy(logits, labels)
//   dlogit = (softmax - onehot) * scale
//   dW += dlogit^T . h ; db += sum dlogit          (fp32 atomics into the grad buffer)
//   dZ    = (dlogit . W) * inv_keep * (h > 0)      (grad w.r.t. the pre-activation of h)
//   db_h += sum_rows dZ                             (bias grad of the layer producing h)
//
// One wave owns one batch row at a time; each lane holds K/64 consecutive
// features of the row.  The 10 logits are 10 wave reductions; softmax runs on
// wave-uniform values; dW partials are summed in LDS (ds_add_f32) across the rows of a
// workgroup and flushed to global memory once per workgroup.  Replaces TF's
// MatMul + BiasAdd + SoftmaxCrossEntropyWithLogits + their gradients + the
// ReluGrad of the layer below (SURVEY K01/K02/K03/K07 fused).
#include "common.h"
#include "head.h"

namespace dtfe {

template <int NC, int K>
__global__ __launch_bounds__(256) void head_xent_kernel(HeadArgs a) {
  constexpr int E = K / 64;        // features per lane
  static_assert(E % 8 == 0, "K must be a multiple of 512");
  __shared__ __attribute__((aligned(16))) float wl[NC * K];   // W as f32 (40 KB)
  __shared__ float red[NC * K];    // workgroup combine of dW partials (40 KB)
  __shared__ float redb[K];        // db_h partials
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < NC * K; i += 256) { red[i] = 0.f; wl[i] = bf2f(a.w[i]); }
  for (int i = threadIdx.x; i < K; i += 256) redb[i] = 0.f;
  __syncthreads();
  float bias[NC];
#pragma unroll
  for (int n = 0; n < NC; ++n) bias[n] = a.b ? a.b[n] : 0.f;

  float dbh[E];
#pragma unroll
  for (int i = 0; i < E; ++i) dbh[i] = 0.f;
  float db[NC];
#pragma unroll
  for (int n = 0; n < NC; ++n) db[n] = 0.f;
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
      float s = 0.f;
      const float* wr = wl + n * K + lane * E;
#pragma unroll
      for (int i = 0; i < E; ++i) s = fmaf(h[i], wr[i], s);
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
#pragma unroll
    for (int n = 0; n < NC; ++n) {
      const float p = __expf(logit[n] - lse);
      dl[n] = (p - (n == label ? 1.f : 0.f)) * a.scale;
      db[n] += dl[n];
      if (a.logits_out && lane == 0) a.logits_out[(long)row * NC + n] = logit[n];
    }
    float lg_label = 0.f;
#pragma unroll
    for (int n = 0; n < NC; ++n) if (n == label) lg_label = logit[n];
    loss_acc += lse - lg_label;
    correct += (am == label);

    // dZ and the dW partials
    u32x4_t outv[E / 8];
#pragma unroll
    for (int i = 0; i < E; ++i) {
      float g = 0.f;
#pragma unroll
      for (int n = 0; n < NC; ++n) {
        g = fmaf(dl[n], wl[n * K + lane * E + i], g);
        atomicAdd(&red[n * K + lane * E + i], dl[n] * h[i]);  // ds_add_f32
      }
      g = h[i] > 0.f ? g * a.inv_keep : 0.f;
      dbh[i] += g;
      reinterpret_cast<bf16*>(&outv[i / 8])[i % 8] = f2bf(g);
    }
#pragma unroll
    for (int c = 0; c < E / 8; ++c)
      *reinterpret_cast<u32x4_t*>(a.dz + (long)row * K + lane * E + c * 8) = outv[c];
  }

#pragma unroll
  for (int i = 0; i < E; ++i) atomicAdd(&redb[lane * E + i], dbh[i]);
  __syncthreads();
  for (int i = threadIdx.x; i < NC * K; i += 256) atomicAdd(a.dw + i, red[i]);
  if (a.dbh)
    for (int i = threadIdx.x; i < K; i += 256) atomicAdd(a.dbh + i, redb[i]);
  if (lane == 0) {
    if (a.db)
#pragma unroll
      for (int n = 0; n < NC; ++n) atomicAdd(a.db + n, db[n]);
    if (a.loss_sum) atomicAdd(a.loss_sum, loss_acc);
    if (a.correct) atomicAdd(a.correct, correct);
  }
}

void launch_head_xent(const HeadArgs& a, hipStream_t s) {
  if (a.NC != 10 || a.K != 1024) throw std::runtime_error("head_xent: only NC=10, K=1024 instantiated");
  int rows_per_wave = a.B >= 2048 ? 8 : (a.B >= 512 ? 4 : 1);
  int blocks = (a.B + 4 * rows_per_wave - 1) / (4 * rows_per_wave);
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL((head_xent_kernel<10, 1024>), dim3(blocks), dim3(256), 0, s, a);
}

}  // namespace dtfe
