// Fused multi-tensor apply_gradients: one launch updates
// every parameter of a model in the flat fp32 master buffer with TF1-exact
// math, refreshes the bf16 working copies the MFMA kernels read (natural and,
// where a backward GEMM wants it, transposed through an LDS tile), and - in
// its last workgroup - advances global_step and Adam's beta powers, the
// scalars TF keeps as separate variables (AssignAdd / _finish in TF1).
//
// TF1 reference semantics (tensorflow/python/training/*.py @ 1.11):
//   SGD       : v -= lr*g
//   Momentum  : a = m*a + g ; v -= lr*a
//   Adam      : lr_t = lr*sqrt(1-b2^t)/(1-b1^t); m = b1 m + (1-b1) g;
//               v2 = b2 v2 + (1-b2) g^2; v -= lr_t * m / (sqrt(v2) + eps)
//   RMSProp   : ms = rho ms + (1-rho) g^2 ; mom = mu mom + lr g / sqrt(ms + eps); v -= mom
//               (ms slot initialised to ONES by the host)
#include "optim.h"

namespace dtfe {

struct Hyper {
  float lr_t;
};

__device__ __forceinline__ float update_one(const OptArgs& a, float lr_t, long i, float g) {
  float v = a.p[i];
  switch (a.kind) {
    case OPT_SGD:
      v -= a.lr * g;
      break;
    case OPT_MOMENTUM: {
      const float acc = a.s1[i] * a.momentum + g;
      a.s1[i] = acc;
      v -= a.lr * acc;
      break;
    }
    case OPT_ADAM: {
      const float m = a.s1[i] * a.beta1 + (1.f - a.beta1) * g;
      const float v2 = a.s2[i] * a.beta2 + (1.f - a.beta2) * g * g;
      a.s1[i] = m;
      a.s2[i] = v2;
      v -= lr_t * m / (sqrtf(v2) + a.eps);
      break;
    }
    case OPT_RMSPROP: {
      const float ms = a.s1[i] * a.rho + (1.f - a.rho) * g * g;
      const float mom = a.s2[i] * a.momentum + a.lr * g / sqrtf(ms + a.eps);
      a.s1[i] = ms;
      a.s2[i] = mom;
      v -= mom;
      break;
    }
  }
  a.p[i] = v;
  return v;
}

__device__ __forceinline__ float load_grad(const OptArgs& a, long i) {
  return (a.g ? a.g[i] : bf2f(a.g16[i])) * a.gscale;
}

__global__ __launch_bounds__(256) void apply_gradients_kernel(OptArgs a) {
  __shared__ bf16 tile[64][66];
  float lr_t = a.lr;
  if (a.kind == OPT_ADAM) {
    const float b1p = a.beta_pow[0], b2p = a.beta_pow[1];
    lr_t = a.lr * sqrtf(1.f - b2p) / (1.f - b1p);
  }
  for (int wi = blockIdx.x; wi < a.nwork; wi += gridDim.x) {
    const OptWork w = a.work[wi];
    const OptSeg sg = a.segs[w.seg];
    if (w.kind == 0) {
      for (long j = threadIdx.x; j < w.count; j += 256) {
        const long li = w.start + j, i = sg.off + li;
        const float v = update_one(a, lr_t, i, load_grad(a, i));
        if (sg.w16) sg.w16[li] = f2bf(v);
      }
    } else {
      // 64x64 tile of tap t: rows r0.., cols c0.. of the [R][C] slice
      const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
      for (int rr = ty; rr < 64; rr += 4) {
        const int r = w.r0 + rr, c = w.c0 + tx;
        if (r < sg.R && c < sg.C) {
          const long li = ((long)r * sg.T + w.t) * sg.C + c, i = sg.off + li;
          const float v = update_one(a, lr_t, i, load_grad(a, i));
          const bf16 b = f2bf(v);
          if (sg.w16) sg.w16[li] = b;
          tile[rr][tx] = b;
        }
      }
      __syncthreads();
      for (int cc = ty; cc < 64; cc += 4) {
        const int c = w.c0 + cc, r = w.r0 + tx;
        if (r < sg.R && c < sg.C) sg.wt16[((long)c * sg.T + w.t) * sg.R + r] = tile[tx][cc];
      }
      __syncthreads();
    }
  }
  // last workgroup: advance the non-slot scalars (every workgroup has read them)
  if (threadIdx.x == 0) {
    __threadfence();
    const uint32_t prev = atomicAdd(a.done_counter, 1u);
    if (prev == gridDim.x - 1) {
      if (a.kind == OPT_ADAM) {
        a.beta_pow[0] *= a.beta1;
        a.beta_pow[1] *= a.beta2;
      }
      if (a.global_step && a.gs_inc) atomicAdd(a.global_step, a.gs_inc);
      atomicExch(a.done_counter, 0u);
      __threadfence();
    }
  }
}

void launch_apply_gradients(const OptArgs& a, hipStream_t s) {
  int blocks = a.nwork < 2048 ? a.nwork : 2048;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(apply_gradients_kernel, dim3(blocks), dim3(256), 0, s, a);
}

}  // namespace dtfe
