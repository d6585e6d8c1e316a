#pragma once
#include "common.h"
#include <stdexcept>
#include <type_traits>

namespace dtfe {

struct HeadArgs {
  int B, NC, K;
  const bf16* h; const bf16* w; const float* b; const int32_t* labels;
  float scale;        // d(loss)/d(logit) scale: 1 / batch
  float inv_keep;     // dropout scale of h (1 when no dropout)
  bf16* dz;           // [B][K]
  bf16* dl; int ld_dl;  // d(loss)/d(logit) rows, bf16 [B][ld_dl]
  float* loss_sum; int32_t* correct; float* logits_out;
  // optional: advanced by one (one thread of workgroup 0) - the per-step sampling / dropout
  // counter of the fused MNIST step, whose readers (the conv1 gather, fc1 dropout) all run
  // before this kernel: one plain increment instead of a grid-wide last-arriver atomic
  int64_t* step_counter;
  // optional: per-workgroup partials instead of the loss / hit atomics - workgroup g stores its
  // loss sum at parts[g] and its hit count at parts[gridDim.x + g] ((B + 3) / 4 workgroups); the
  // head weight gradient's bias workgroup folds them into loss_sum / correct (HeadWgradArgs.parts).
  // 256 same-address atomics per launch cost ~2.5 us of the kernel's 7.8 (bench/cnn_kernels.py
  // head vs head_noacc); the fold is also a fixed-order, bitwise-reproducible sum.
  float* parts;
};

void launch_head_xent(const HeadArgs& a, hipStream_t s);

// The same per-row head at fp32 (the `--dtype fp32` CNN step): fp32 h / W / b in, fp32 logits
// (optional), dlogit rows [B][NC] (the head weight-gradient GEMM's operand) and dZ [B][K] out;
// loss / hits by one atomic per workgroup; step_counter as above.  Every product and sum is an
// fp32 FMA / add (the dot products as lane-strided fmaf chains + a butterfly).
struct HeadF32Args {
  int B, NC, K;
  const float* h; const float* w; const float* b; const int32_t* labels;
  float scale, inv_keep;
  float* dz; float* dl; float* logits_out;
  float* loss_sum; int32_t* correct;
  int64_t* step_counter;
};
// false: shape not instantiated (NC = 10, K = 1024 only)
bool launch_head_xent_f32(const HeadF32Args& a, hipStream_t s);

// dW[c][k] = scale * sum_b dl[b][c] h[b][k] (row stride ldw), db[c] = scale * sum_b dl[b][c];
// stored, not accumulated (one workgroup per 16 columns, fixed summation order)
struct HeadWgradArgs {
  int B, NC, K;
  const bf16* dl; int ld_dl;   // [B][ld_dl]
  const bf16* h; int ldh;      // [B][ldh]
  float* dw; int ldw;          // [NC][ldw]
  float* db;                   // [NC] (optional)
  float scale;
  // optional: head_xent's per-workgroup loss / hit partials (2 x nparts floats), summed in a fixed
  // order by the bias workgroup and added to loss_sum / correct (one plain read-modify-write)
  const float* parts; int nparts; float* loss_sum; int32_t* correct;
};
void launch_head_wgrad(const HeadWgradArgs& a, hipStream_t s);

// Bias workgroup: loss_sum += sum(parts[0:n]), correct += sum(parts[n:2n]) (wave 0, lane-strided
// partial sums, then a butterfly: lane 0's total has a fixed summation order)
__device__ __forceinline__ void head_fold_parts(const HeadWgradArgs& a) {
  if (!a.parts || threadIdx.x >= 64) return;
  const int lane = threadIdx.x;
  float l = 0.f, c = 0.f;
  for (int i = lane; i < a.nparts; i += 64) {
    l += a.parts[i];
    c += a.parts[a.nparts + i];
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    l += __shfl_xor(l, o, 64);
    c += __shfl_xor(c, o, 64);
  }
  if (lane == 0) {
    *a.loss_sum += l;
    *a.correct += (int)c;
  }
}

// Workgroup `bid` (256 threads) of the head weight gradient: columns 8*bid..+7 of dW for the whole
// batch (bid == K/8: the bias); red: 4 x 80 floats of LDS.  See head.hip.
template <int NC, int ROWS>
__device__ __forceinline__ void head_wgrad_body(const HeadWgradArgs& a, int bid, float (*red)[NC * 8]) {
  static_assert(NC * 8 == 80, "the butterfly below is laid out for 10 classes x 8 columns");
  constexpr int V = NC * 8;
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const bool bias_blk = bid * 8 >= a.K;
  const int col0 = bid * 8;
  u32x4_t hv[ROWS], d0[ROWS], d1[ROWS];
#pragma unroll
  for (int i = 0; i < ROWS; ++i) {
    const int b = t + 256 * i;
    const bool ok = b < a.B;
    hv[i] = (ok && !bias_blk) ? *reinterpret_cast<const u32x4_t*>(a.h + (long)b * a.ldh + col0) : u32x4_t{0u, 0u, 0u, 0u};
    d0[i] = ok ? *reinterpret_cast<const u32x4_t*>(a.dl + (long)b * a.ld_dl) : u32x4_t{0u, 0u, 0u, 0u};
    d1[i] = ok ? *reinterpret_cast<const u32x4_t*>(a.dl + (long)b * a.ld_dl + 8) : u32x4_t{0u, 0u, 0u, 0u};
  }
  float v[V];
#pragma unroll
  for (int j = 0; j < V; ++j) v[j] = 0.f;
#pragma unroll
  for (int i = 0; i < ROWS; ++i) {
    float h[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) h[e] = bias_blk ? ((t + 256 * i) < a.B ? 1.f : 0.f) : bf2f((bf16)(hv[i][e >> 1] >> (16 * (e & 1))));
#pragma unroll
    for (int n = 0; n < NC; ++n) {
      const uint32_t w = n < 8 ? d0[i][n >> 1] : d1[i][(n - 8) >> 1];
      const float d = bf2f((bf16)(w >> (16 * (n & 1))));
#pragma unroll
      for (int e = 0; e < 8; ++e) v[n * 8 + e] = fmaf(d, h[e], v[n * 8 + e]);
    }
  }
  // halving butterfly over lane bits 5..2: 80 -> 40 -> 20 -> 10 -> 5 values per lane
  auto halve = [&](auto half_c, int mask) {
    constexpr int H = decltype(half_c)::value;
    const bool hi = (lane & mask) != 0;
#pragma unroll
    for (int j = 0; j < H; ++j) {
      const float send = hi ? v[j] : v[H + j];
      const float keep = hi ? v[H + j] : v[j];
      v[j] = keep + __shfl_xor(send, mask, 64);
    }
  };
  halve(std::integral_constant<int, 40>{}, 32);
  halve(std::integral_constant<int, 20>{}, 16);
  halve(std::integral_constant<int, 10>{}, 8);
  halve(std::integral_constant<int, 5>{}, 4);
#pragma unroll
  for (int j = 0; j < 5; ++j) {
    v[j] += __shfl_xor(v[j], 2, 64);
    v[j] += __shfl_xor(v[j], 1, 64);
  }
  // lane holds values ((b5 ? 40 : 0) + (b4 ? 20 : 0) + (b3 ? 10 : 0) + (b2 ? 5 : 0) + j)
  if ((lane & 3) == 0) {
    const int base = ((lane >> 5) & 1) * 40 + ((lane >> 4) & 1) * 20 + ((lane >> 3) & 1) * 10 + ((lane >> 2) & 1) * 5;
#pragma unroll
    for (int j = 0; j < 5; ++j) red[wid][base + j] = v[j];
  }
  __syncthreads();
  if (t < V) {
    const float s = ((red[0][t] + red[1][t]) + red[2][t]) + red[3][t];
    const int n = t >> 3, e = t & 7;
    if (!bias_blk) a.dw[(long)n * a.ldw + col0 + e] = s * a.scale;
    else if (e == 0) a.db[n] = s * a.scale;
  }
  if (bias_blk) head_fold_parts(a);
}

// The grouped fc-backward launch's head piece (gemm_dense.hip): 4 columns of dW per workgroup
// (bid == K/4: the bias) with the rows streamed one 256-row pass at a time - 40 accumulators, so
// the piece stays inside the GEMM pieces' register budget (the 8-column body above set the grouped
// kernel to 148 VGPRs).  red: 4 x 40 floats of LDS.
template <int NC>
__device__ __forceinline__ void head_wgrad4_body(const HeadWgradArgs& a, int bid, float (*red)[NC * 4]) {
  static_assert(NC * 4 == 40, "the butterfly below is laid out for 10 classes x 4 columns");
  constexpr int V = NC * 4;
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const bool bias_blk = bid * 4 >= a.K;
  const int col0 = bias_blk ? 0 : bid * 4;
  float v[V];
#pragma unroll
  for (int j = 0; j < V; ++j) v[j] = 0.f;
#pragma unroll 1
  for (int b0 = 0; b0 < a.B; b0 += 256) {
    const int b = b0 + t;
    const bool ok = b < a.B;
    const long r = ok ? b : 0;  // clamped row: loads stay in bounds, the products are zeroed
    const u32x2_t hv = *reinterpret_cast<const u32x2_t*>(a.h + r * a.ldh + col0);
    const u32x4_t d0 = *reinterpret_cast<const u32x4_t*>(a.dl + r * a.ld_dl);
    const uint32_t d1 = *reinterpret_cast<const uint32_t*>(a.dl + r * a.ld_dl + 8);
    float h[4];
#pragma unroll
    for (int e = 0; e < 4; ++e)
      h[e] = !ok ? 0.f : bias_blk ? 1.f : bf2f((bf16)(hv[e >> 1] >> (16 * (e & 1))));
#pragma unroll
    for (int n = 0; n < NC; ++n) {
      const uint32_t w = n < 8 ? d0[n >> 1] : d1;
      const float d = bf2f((bf16)(w >> (16 * (n & 1))));
#pragma unroll
      for (int e = 0; e < 4; ++e) v[n * 4 + e] = fmaf(d, h[e], v[n * 4 + e]);
    }
  }
  // halving butterfly over lane bits 5..3: 40 -> 20 -> 10 -> 5 values per lane, then bits 2..0
  auto halve = [&](auto half_c, int mask) {
    constexpr int H = decltype(half_c)::value;
    const bool hi = (lane & mask) != 0;
#pragma unroll
    for (int j = 0; j < H; ++j) {
      const float send = hi ? v[j] : v[H + j];
      const float keep = hi ? v[H + j] : v[j];
      v[j] = keep + __shfl_xor(send, mask, 64);
    }
  };
  halve(std::integral_constant<int, 20>{}, 32);
  halve(std::integral_constant<int, 10>{}, 16);
  halve(std::integral_constant<int, 5>{}, 8);
#pragma unroll
  for (int j = 0; j < 5; ++j) {
    v[j] += __shfl_xor(v[j], 4, 64);
    v[j] += __shfl_xor(v[j], 2, 64);
    v[j] += __shfl_xor(v[j], 1, 64);
  }
  // lane holds values ((b5 ? 20 : 0) + (b4 ? 10 : 0) + (b3 ? 5 : 0) + j)
  if ((lane & 7) == 0) {
    const int base = ((lane >> 5) & 1) * 20 + ((lane >> 4) & 1) * 10 + ((lane >> 3) & 1) * 5;
#pragma unroll
    for (int j = 0; j < 5; ++j) red[wid][base + j] = v[j];
  }
  __syncthreads();
  if (t < V) {
    const float s = ((red[0][t] + red[1][t]) + red[2][t]) + red[3][t];
    const int n = t >> 2, e = t & 3;
    if (!bias_blk) a.dw[(long)n * a.ldw + col0 + e] = s * a.scale;
    else if (e == 0) a.db[n] = s * a.scale;
  }
  if (bias_blk) head_fold_parts(a);
}

// The GAN discriminator's output layer with both GAN losses and their gradients down to the hidden
// layer, one launch (reference gan/distributed_gan.py:128-143): for the B real rows
// and B fake rows of d1 = relu(.) [2B][DH]: p = sigmoid(d1 . Wd2 + bd2); gen_loss = -mean(log p_fake),
// disc_loss = -mean(log p_real + log(1 - p_fake)) (no epsilon unless clamp_eps > 0, as gan_loss);
// dlog = d disc_loss / d logit [2B], dlog_g = d gen_loss / d logit_fake [B]; dWd2 = d1^T dlog, dbd2 =
// sum dlog (stored); dd1 = dlog Wd2^T * relu'(d1) [2B][DH]; ddf = dlog_g Wd2^T * relu'(d1_fake) [B][DH].
// Replaces the N = 1 GEMM, gan_loss, the dWd2 GEMM and the two K = 1 GEMMs (5 launches).  One wave per
// (real, fake) row pair; per-workgroup partials (write-through) + ticket, the last workgroup sums them in
// workgroup order: every output is bitwise reproducible.
struct GanHeadArgs {
  int B, DH;
  const float* d1; const float* w; const float* b;
  float* p; float* dlog; float* dlog_g;     // optional outputs ([2B], [2B], [B])
  float* gw; float* gb;                     // dWd2 [DH], dbd2 [1] (stored)
  float* dd1; float* ddf;                   // [2B][DH], [B][DH]
  float* gen_loss; float* disc_loss;        // stored
  float clamp_eps;
  float* ws;                                // gan_head_ws_floats(B, DH) floats, zeroed once
};
long gan_head_ws_floats(int B, int DH);
// false: DH > 256 or DH % 4 (the caller runs the unfused chain)
bool launch_gan_disc_head(const GanHeadArgs& a, hipStream_t s);

}  // namespace dtfe
