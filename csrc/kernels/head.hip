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
#include "gemm_dense.h"

#include <algorithm>
#include <type_traits>

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
    const float l = red_loss[0] + red_loss[1] + red_loss[2] + red_loss[3];
    const int c = red_correct[0] + red_correct[1] + red_correct[2] + red_correct[3];
    if (a.parts) {  // folded by the head weight gradient's bias workgroup (head.h)
      a.parts[blockIdx.x] = l;
      a.parts[gridDim.x + blockIdx.x] = (float)c;
    } else {
      if (a.loss_sum) atomicAdd(a.loss_sum, l);
      if (a.correct) atomicAdd(a.correct, c);
    }
  }
}

// fp32 head: one wave per row as above; the wave's W slice (NC x K/64 fp32, 160 VGPRs for 10 x 16)
// and h row go straight to registers (16-B loads); replaces the fp32 step's head GEMM + softmax-xent
// + dlogit . W GEMM + step-counter increment (four launches, ~54 us, profiles/r6_fp32_rows.txt)
template <int NC, int K>
__global__ __launch_bounds__(256) void head_xent_f32_kernel(HeadF32Args a) {
  constexpr int E = K / 64;
  static_assert(E % 4 == 0, "K must be a multiple of 256");
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  __shared__ float red_loss[4];
  __shared__ int red_correct[4];
  if (a.step_counter && blockIdx.x == 0 && threadIdx.x == 0) *a.step_counter += 1;
  const int row = min(blockIdx.x * 4 + wid, a.B - 1);
  const bool live = blockIdx.x * 4 + wid < a.B;
  f32x4_t wv[NC][E / 4], hv[E / 4];
#pragma unroll
  for (int c = 0; c < E / 4; ++c) hv[c] = *reinterpret_cast<const f32x4_t*>(a.h + (long)row * K + lane * E + c * 4);
#pragma unroll
  for (int n = 0; n < NC; ++n)
#pragma unroll
    for (int c = 0; c < E / 4; ++c) wv[n][c] = *reinterpret_cast<const f32x4_t*>(a.w + (long)n * K + lane * E + c * 4);
  const int label = a.labels[row];
  float logit[NC];
#pragma unroll
  for (int n = 0; n < NC; ++n) {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < E; ++i) s = fmaf(hv[i / 4][i % 4], wv[n][i / 4][i % 4], s);
    logit[n] = s;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1)
#pragma unroll
    for (int n = 0; n < NC; ++n) logit[n] += __shfl_xor(logit[n], o, 64);
#pragma unroll
  for (int n = 0; n < NC; ++n) logit[n] += a.b ? a.b[n] : 0.f;
  float mx = logit[0];
  int am = 0;
#pragma unroll
  for (int n = 1; n < NC; ++n) if (logit[n] > mx) { mx = logit[n]; am = n; }
  float se = 0.f;
#pragma unroll
  for (int n = 0; n < NC; ++n) se += expf(logit[n] - mx);
  const float lse = mx + logf(se);
  float dl[NC], lg_label = 0.f;
#pragma unroll
  for (int n = 0; n < NC; ++n) {
    const float p = expf(logit[n] - lse);
    dl[n] = (p - (n == label ? 1.f : 0.f)) * a.scale;
    if (n == label) lg_label = logit[n];
  }
  if (live && lane < NC) {
    float v = 0.f, lv = 0.f;
#pragma unroll
    for (int n = 0; n < NC; ++n) if (n == lane) { v = dl[n]; lv = logit[n]; }
    a.dl[(long)row * NC + lane] = v;
    if (a.logits_out) a.logits_out[(long)row * NC + lane] = lv;
  }
#pragma unroll
  for (int c = 0; c < E / 4; ++c) {
    f32x4_t o;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float g = 0.f;
#pragma unroll
      for (int n = 0; n < NC; ++n) g = fmaf(dl[n], wv[n][c][j], g);
      o[j] = hv[c][j] > 0.f ? g * a.inv_keep : 0.f;
    }
    if (live) *reinterpret_cast<f32x4_t*>(a.dz + (long)row * K + lane * E + c * 4) = o;
  }
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

bool launch_head_xent_f32(const HeadF32Args& a, hipStream_t s) {
  if (a.NC != 10 || a.K != 1024 || a.B < 1) return false;
  hipLaunchKernelGGL((head_xent_f32_kernel<10, 1024>), dim3((a.B + 3) / 4), dim3(256), 0, s, a);
  return true;
}

void launch_head_xent(const HeadArgs& a, hipStream_t s) {
  if (a.NC != 10 || a.K != 1024) throw std::runtime_error("head_xent: only NC=10, K=1024 instantiated");
  const int blocks = (a.B + 3) / 4;  // one row per wave
  hipLaunchKernelGGL((head_xent_kernel<10, 1024>), dim3(blocks), dim3(256), 0, s, a);
}

}  // namespace dtfe

namespace dtfe {

// Classifier-head weight / bias gradient: dW[c][k] = sum_b dl[b][c] h[b][k], db[c] = sum_b dl[b][c].
// The layer is 10 x 1024 over a 1024-row batch (21 MFLOP, 2 MB of h).  One 256-thread workgroup
// owns 8 columns of dW for the whole batch (128 workgroups + one for the bias): a thread loads
// the 16-B h chunk and the dlogit row of each of its rows (all loads in flight at once),
// accumulates 10 x 8 partial sums, and the wave reduces them with a halving butterfly - each
// exchange step sends half of the lane's remaining values, 85 shuffles instead of 80 x 6 - to
// 16 lanes holding 5 totals each; the 4 waves are summed in order through LDS.  Fixed
// summation order (bitwise reproducible), no atomics, no cross-workgroup reduction.  (The
// previous form - 64 workgroups of 1024 threads, 16 columns each, a 64-step serial LDS sum per
// output - took ~11 us on the MNIST step's critical path.)
template <int NC, int ROWS>
__global__ __launch_bounds__(256) void head_wgrad_kernel(HeadWgradArgs a) {
  __shared__ float red[4][NC * 8];
  head_wgrad_body<NC, ROWS>(a, blockIdx.x, red);
}

void launch_head_wgrad(const HeadWgradArgs& a, hipStream_t s) {
  if (a.NC != 10 || a.K % 8 || a.ld_dl < 16 || a.ld_dl % 8 || a.ldh % 8 || a.B > 1024)
    throw std::runtime_error("head_wgrad: needs NC=10, K % 8 == 0, 16-B aligned dl rows of >= 16 and h rows, B <= 1024");
  if (a.parts && (!a.db || !a.loss_sum || !a.correct))
    throw std::runtime_error("head_wgrad: folding the loss partials needs db (the bias workgroup), loss_sum and correct");
  if (glds_group_record_head(a)) return;  // recorded into a grouped launch (gemm_dense.hip)
  const int blocks = a.K / 8 + (a.db ? 1 : 0);
  if (a.B <= 256) hipLaunchKernelGGL((head_wgrad_kernel<10, 1>), dim3(blocks), dim3(256), 0, s, a);
  else if (a.B <= 512) hipLaunchKernelGGL((head_wgrad_kernel<10, 2>), dim3(blocks), dim3(256), 0, s, a);
  else hipLaunchKernelGGL((head_wgrad_kernel<10, 4>), dim3(blocks), dim3(256), 0, s, a);
}

namespace {
constexpr int GH_SLOT = 256 + 4;  // per-workgroup partial: dWd2[256], dbd2, gen, disc, pad
int gan_head_grid(int B) { return std::max(1, std::min(256, (B + 3) / 4)); }
}  // namespace

long gan_head_ws_floats(int B, int DH) { (void)DH; return (long)gan_head_grid(B) * GH_SLOT + 4; }

__global__ __launch_bounds__(256) void gan_disc_head_kernel(GanHeadArgs a) {
  __shared__ float red[4][GH_SLOT];
  __shared__ int lastf;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, DH = a.DH, B = a.B;
  const bool on = 4 * lane < DH;  // this lane's 4 columns
  const int c0 = on ? 4 * lane : 0;
  const f32x4_t zero = {0.f, 0.f, 0.f, 0.f};
  const f32x4_t wv = on ? *reinterpret_cast<const f32x4_t*>(a.w + c0) : zero;
  const float bias = a.b ? a.b[0] : 0.f, invB = 1.f / (float)B;
  f32x4_t gw = zero;
  float gb = 0.f, gl = 0.f, dl = 0.f;  // (lane-uniform)
  for (int i = blockIdx.x * 4 + wid; i < B; i += gridDim.x * 4) {
    const f32x4_t xr = on ? *reinterpret_cast<const f32x4_t*>(a.d1 + (long)i * DH + c0) : zero;
    const f32x4_t xf = on ? *reinterpret_cast<const f32x4_t*>(a.d1 + (long)(B + i) * DH + c0) : zero;
    float zr = 0.f, zf = 0.f;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      zr = __builtin_fmaf(xr[e], wv[e], zr);
      zf = __builtin_fmaf(xf[e], wv[e], zf);
    }
    zr = wave_sum(zr) + bias;
    zf = wave_sum(zf) + bias;
    const float pr = sigmoidf_(zr), pf = sigmoidf_(zf);
    float pr_c = pr, pf_c = pf, qf_c = 1.f - pf;
    if (a.clamp_eps > 0.f) {
      pr_c = fmaxf(pr, a.clamp_eps);
      pf_c = fmaxf(pf, a.clamp_eps);
      qf_c = fmaxf(1.f - pf, a.clamp_eps);
    }
    gl += -logf(pf_c);
    dl += -(logf(pr_c) + logf(qf_c));
    // d/dz of -log(sigmoid(z)) = -(1 - s);  d/dz of -log(1 - sigmoid(z)) = s
    const float gr = -(1.f - pr) * invB, gf = pf * invB, gg = -(1.f - pf) * invB;
    if (lane == 0) {
      if (a.p) { a.p[i] = pr; a.p[B + i] = pf; }
      if (a.dlog) { a.dlog[i] = gr; a.dlog[B + i] = gf; }
      if (a.dlog_g) a.dlog_g[i] = gg;
    }
    if (on) {
      f32x4_t orr, off, ogg;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float mr = xr[e] > 0.f ? wv[e] : 0.f, mf = xf[e] > 0.f ? wv[e] : 0.f;  // Wd2 * relu'(d1)
        orr[e] = gr * mr;
        off[e] = gf * mf;
        ogg[e] = gg * mf;
        gw[e] = __builtin_fmaf(xf[e], gf, __builtin_fmaf(xr[e], gr, gw[e]));
      }
      *reinterpret_cast<f32x4_t*>(a.dd1 + (long)i * DH + c0) = orr;
      *reinterpret_cast<f32x4_t*>(a.dd1 + (long)(B + i) * DH + c0) = off;
      *reinterpret_cast<f32x4_t*>(a.ddf + (long)i * DH + c0) = ogg;
    }
    gb += gr + gf;
  }
  // workgroup partial (waves summed in order) -> write-through slab, ticket; the last arriver sums the
  // slabs in workgroup order (the split-K hand-off of gemm_dense.h)
  if (on) *reinterpret_cast<f32x4_t*>(&red[wid][c0]) = gw;
  if (lane == 0) { red[wid][256] = gb; red[wid][257] = gl; red[wid][258] = dl; }
  __syncthreads();
  const int t = threadIdx.x;
  const __amdgpu_buffer_rsrc_t slab =
      __builtin_amdgcn_make_buffer_rsrc(a.ws + (long)blockIdx.x * GH_SLOT, (short)0, GH_SLOT * 4, 0x00020000);
  for (int k = t; k < GH_SLOT; k += 256) {
    const float v = ((red[0][k] + red[1][k]) + red[2][k]) + red[3][k];
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), slab, k * 4, 0, 16);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  int* ctr = reinterpret_cast<int*>(a.ws + (long)gridDim.x * GH_SLOT);
  if (t == 0) {
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
  const int G = gridDim.x;
  for (int k = t; k < 259; k += 256) {
    if (k >= DH && k < 256) continue;
    // the slabs' column k in workgroup order, 16 loads in flight per chunk (a serial load chain here
    // cost ~10 us)
    float sum = 0.f;
    for (int g0 = 0; g0 < G; g0 += 16) {
      float v[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) v[j] = g0 + j < G ? a.ws[(long)(g0 + j) * GH_SLOT + k] : 0.f;
#pragma unroll
      for (int j = 0; j < 16; ++j) sum += v[j];
    }
    if (k < 256) a.gw[k] = sum;
    else if (k == 256) { if (a.gb) a.gb[0] = sum; }
    else if (k == 257) *a.gen_loss = sum * invB;
    else *a.disc_loss = sum * invB;
  }
}

bool launch_gan_disc_head(const GanHeadArgs& a, hipStream_t s) {
  if (a.DH > 256 || a.DH % 4 || a.B < 1 || !a.ws || !a.gw || !a.dd1 || !a.ddf) return false;
  hipLaunchKernelGGL(gan_disc_head_kernel, dim3(gan_head_grid(a.B)), dim3(256), 0, s, a);
  return true;
}

}  // namespace dtfe
