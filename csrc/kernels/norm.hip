// BatchNorm (training), option-A residual shortcuts, global average pool and
// 3x3/s2 max pool for the ResNet models - see norm.h.
//
// Layout: NHWC bf16 viewed as [R][C] rows with C % 8 == 0 and C/8 a power of
// two; every thread owns one 16-byte chunk (8 channels) of a row, so loads and
// stores are 16 B vectors and a warp-wide load covers whole 128 B lines.
// Channel statistics are reduced per workgroup through LDS and then added to
// the [2][C] accumulators with one atomic per channel and workgroup.
#include "norm.h"

#include <stdexcept>

namespace dtfe {

namespace {

constexpr int NT = 256;

__device__ __forceinline__ void unpack8(const u32x4_t v, float (&f)[8]) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = bf2f((bf16)(v[i] & 0xffffu));
    f[2 * i + 1] = bf2f((bf16)(v[i] >> 16));
  }
}

__device__ __forceinline__ u32x4_t pack8(const float (&f)[8]) {
  u32x4_t v;
#pragma unroll
  for (int i = 0; i < 4; ++i) v[i] = pack_bf16x2(f[2 * i], f[2 * i + 1]);
  return v;
}

__device__ __forceinline__ float act_fwd(float x, int act) { return apply_act(x, act); }

// per-thread (row slot, chunk) decomposition of a block of NT threads
struct Slots {
  int tpr, rpp, chunk, slot;
  __device__ Slots(int C) {
    tpr = C / 8;
    rpp = NT / tpr;
    chunk = threadIdx.x % tpr;
    slot = threadIdx.x / tpr;
  }
};

// block-reduce s[8], q[8] of every thread onto channels and add them to stats[0..C), stats[C..2C)
__device__ void reduce_stats(const float (&s)[8], const float (&q)[8], int C, float* stats) {
  extern __shared__ float red[];  // [rpp][2][C]
  const Slots S(C);
  float* mine = red + S.slot * 2 * C;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    mine[S.chunk * 8 + e] = s[e];
    mine[C + S.chunk * 8 + e] = q[e];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < 2 * C; c += NT) {
    float v = 0.f;
    for (int r = 0; r < S.rpp; ++r) v += red[r * 2 * C + c];
    atomicAdd(stats + c, v);
  }
}

// Statistics are accumulated around a per-channel shift K = x[row 0][c] (sum (x-K), sum (x-K)^2):
// the one-pass E[x^2] - E[x]^2 form loses the variance to cancellation when |mean| >> std.
__global__ __launch_bounds__(NT) void bn_stats_kernel(BnArgs a) {
  const Slots S(a.C);
  float k[8];
  unpack8(*reinterpret_cast<const u32x4_t*>(a.x + S.chunk * 8), k);
  float s[8] = {}, q[8] = {};
  for (long r = (long)blockIdx.x * S.rpp + S.slot; r < a.R; r += (long)gridDim.x * S.rpp) {
    float f[8];
    unpack8(*reinterpret_cast<const u32x4_t*>(a.x + r * a.C + S.chunk * 8), f);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float d = f[e] - k[e];
      s[e] += d;
      q[e] += d * d;
    }
  }
  reduce_stats(s, q, a.C, a.stats);
}

__device__ __forceinline__ void chan_params(const BnArgs& a, int c, float& mean, float& invstd) {
  const float inv_r = 1.f / (float)a.R;
  const float d = a.stats[c] * inv_r;
  mean = bf2f(a.x[c]) + d;
  const float var = fmaxf(a.stats[a.C + c] * inv_r - d * d, 0.f);
  invstd = rsqrtf(var + a.eps);
}

__global__ __launch_bounds__(NT) void bn_apply_kernel(BnArgs a) {
  const Slots S(a.C);
  if (blockIdx.x == 0) {  // saved statistics + moving averages (TF: unbiased batch variance)
    for (int c = threadIdx.x; c < a.C; c += NT) {
      float mean, invstd;
      chan_params(a, c, mean, invstd);
      if (a.mean) a.mean[c] = mean;
      if (a.invstd) a.invstd[c] = invstd;
      if (a.moving_mean) {
        const float var = 1.f / (invstd * invstd) - a.eps;
        const float unb = a.R > 1 ? var * (float)a.R / (float)(a.R - 1) : var;
        a.moving_mean[c] = a.moving_mean[c] * a.momentum + mean * (1.f - a.momentum);
        a.moving_var[c] = a.moving_var[c] * a.momentum + unb * (1.f - a.momentum);
      }
    }
  }
  float scale[8], shift[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int c = S.chunk * 8 + e;
    float mean, invstd;
    chan_params(a, c, mean, invstd);
    scale[e] = a.gamma[c] * invstd;
    shift[e] = a.beta[c] - mean * scale[e];
  }
  const bool res_identity = a.res && a.rstride == 1 && a.RC == a.C && a.RH == a.OH && a.RW == a.OW;
  const bool res_chunk = a.res && S.chunk * 8 < a.RC;
  for (long r = (long)blockIdx.x * S.rpp + S.slot; r < a.R; r += (long)gridDim.x * S.rpp) {
    float f[8];
    unpack8(*reinterpret_cast<const u32x4_t*>(a.x + r * a.C + S.chunk * 8), f);
#pragma unroll
    for (int e = 0; e < 8; ++e) f[e] = f[e] * scale[e] + shift[e];
    if (res_chunk) {
      long ro;
      if (res_identity) {
        ro = r * a.C + S.chunk * 8;
      } else {
        const long hw = (long)a.OH * a.OW, b = r / hw;
        const int p = (int)(r - b * hw), oy = p / a.OW, ox = p - oy * a.OW;
        ro = ((b * a.RH + (long)oy * a.rstride) * a.RW + (long)ox * a.rstride) * a.RC + S.chunk * 8;
      }
      float g[8];
      unpack8(*reinterpret_cast<const u32x4_t*>(a.res + ro), g);
#pragma unroll
      for (int e = 0; e < 8; ++e) f[e] += g[e];
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) f[e] = act_fwd(f[e], a.act);
    *reinterpret_cast<u32x4_t*>(a.out + r * a.C + S.chunk * 8) = pack8(f);
  }
}

// g = dy * act'(y) for 8 channels
__device__ __forceinline__ void masked_grad(const BnArgs& a, long off, float (&g)[8]) {
  unpack8(*reinterpret_cast<const u32x4_t*>(a.dy + off), g);
  if (a.act != ACT_NONE) {
    float y[8];
    unpack8(*reinterpret_cast<const u32x4_t*>(a.y + off), y);
#pragma unroll
    for (int e = 0; e < 8; ++e) g[e] *= act_grad_from_out(y[e], a.act);
  }
}

__global__ __launch_bounds__(NT) void bn_bwd_stats_kernel(BnArgs a) {
  const Slots S(a.C);
  float mean[8], invstd[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    mean[e] = a.mean[S.chunk * 8 + e];
    invstd[e] = a.invstd[S.chunk * 8 + e];
  }
  float s[8] = {}, q[8] = {};
  for (long r = (long)blockIdx.x * S.rpp + S.slot; r < a.R; r += (long)gridDim.x * S.rpp) {
    const long off = r * a.C + S.chunk * 8;
    float g[8], x[8];
    masked_grad(a, off, g);
    unpack8(*reinterpret_cast<const u32x4_t*>(a.x + off), x);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      s[e] += g[e];
      q[e] += g[e] * (x[e] - mean[e]) * invstd[e];
    }
  }
  reduce_stats(s, q, a.C, a.stats);
}

__global__ __launch_bounds__(NT) void bn_bwd_apply_kernel(BnArgs a) {
  const Slots S(a.C);
  if (blockIdx.x == 0) {
    for (int c = threadIdx.x; c < a.C; c += NT) {
      if (a.dbeta) a.dbeta[c] += a.stats[c];
      if (a.dgamma) a.dgamma[c] += a.stats[a.C + c];
    }
  }
  const float inv_r = 1.f / (float)a.R;
  float mean[8], invstd[8], k[8], sg[8], sgx[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int c = S.chunk * 8 + e;
    mean[e] = a.mean[c];
    invstd[e] = a.invstd[c];
    k[e] = a.gamma[c] * invstd[e];
    sg[e] = a.stats[c] * inv_r;
    sgx[e] = a.stats[a.C + c] * inv_r;
  }
  for (long r = (long)blockIdx.x * S.rpp + S.slot; r < a.R; r += (long)gridDim.x * S.rpp) {
    const long off = r * a.C + S.chunk * 8;
    float g[8], x[8], dx[8];
    masked_grad(a, off, g);
    unpack8(*reinterpret_cast<const u32x4_t*>(a.x + off), x);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float xh = (x[e] - mean[e]) * invstd[e];
      dx[e] = k[e] * (g[e] - sg[e] - xh * sgx[e]);
    }
    *reinterpret_cast<u32x4_t*>(a.out + off) = pack8(dx);
    if (a.dres) *reinterpret_cast<u32x4_t*>(a.dres + off) = pack8(g);
  }
}

// workgroups for R rows: `per_thread` rows per thread, at most max_blocks.  The statistics
// kernels use 8 rows per thread (fewer workgroups -> fewer contended per-channel atomics),
// the apply kernels 2 (no atomics: as many workgroups as fill the chip).
int grid_for(long R, int C, int max_blocks, int per_thread) {
  const int rpp = NT / (C / 8);
  long rows_per_block = (long)rpp * per_thread;
  long g = (R + rows_per_block - 1) / rows_per_block;
  if (g > max_blocks) g = max_blocks;
  return g < 1 ? 1 : (int)g;
}

void check(const BnArgs& a) {
  const int t = a.C / 8;
  if (a.C % 8 || t > NT || (t & (t - 1))) throw std::runtime_error("bn: C must be 8 * 2^k <= 2048");
}

__global__ void shortcut_grad_kernel(const bf16* g, bf16* dx, int B, int OH, int OW, int C, int XH, int XW, int XC,
                                     int stride) {
  const int cpr = XC / 8;
  const long n = (long)B * OH * OW * cpr;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const long row = i / cpr;
    const int ch = (int)(i - row * cpr) * 8;
    const long hw = (long)OH * OW, b = row / hw;
    const int p = (int)(row - b * hw), oy = p / OW, ox = p - oy * OW;
    const long xo = ((b * XH + (long)oy * stride) * XW + (long)ox * stride) * XC + ch;
    float a8[8], b8[8];
    unpack8(*reinterpret_cast<const u32x4_t*>(g + row * C + ch), a8);
    unpack8(*reinterpret_cast<const u32x4_t*>(dx + xo), b8);
#pragma unroll
    for (int e = 0; e < 8; ++e) b8[e] += a8[e];
    *reinterpret_cast<u32x4_t*>(dx + xo) = pack8(b8);
  }
}

// one workgroup per image: threads = (chunk, pixel lane); pixel lanes reduce through LDS
__global__ __launch_bounds__(256) void gap_fwd_kernel(const bf16* x, bf16* y, int B, int HW, int C) {
  __shared__ float red[256 * 8];
  const int cpr = C / 8;  // power of two <= 256
  const int lanes = 256 / cpr, chunk = threadIdx.x % cpr, pl = threadIdx.x / cpr;
  const long b = blockIdx.x;
  float s[8] = {};
  for (int p = pl; p < HW; p += lanes) {
    float f[8];
    unpack8(*reinterpret_cast<const u32x4_t*>(x + (b * HW + p) * C + chunk * 8), f);
#pragma unroll
    for (int e = 0; e < 8; ++e) s[e] += f[e];
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) red[threadIdx.x * 8 + e] = s[e];
  __syncthreads();
  if (pl == 0) {
    for (int l = 1; l < lanes; ++l)
#pragma unroll
      for (int e = 0; e < 8; ++e) s[e] += red[(l * cpr + chunk) * 8 + e];
#pragma unroll
    for (int e = 0; e < 8; ++e) s[e] *= 1.f / (float)HW;
    *reinterpret_cast<u32x4_t*>(y + b * C + chunk * 8) = pack8(s);
  }
}

__global__ void gap_bwd_kernel(const bf16* dy, bf16* dx, int B, int HW, int C) {
  const int cpr = C / 8;
  const long n = (long)B * HW * cpr;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const long row = i / cpr;
    const int ch = (int)(i - row * cpr) * 8;
    const long b = row / HW;
    float f[8];
    unpack8(*reinterpret_cast<const u32x4_t*>(dy + b * C + ch), f);
#pragma unroll
    for (int e = 0; e < 8; ++e) f[e] *= 1.f / (float)HW;
    *reinterpret_cast<u32x4_t*>(dx + row * C + ch) = pack8(f);
  }
}

__global__ void maxpool3_fwd_kernel(const bf16* x, bf16* y, uint8_t* am, int B, int H, int W, int C, int OH,
                                    int OW) {
  const long n = (long)B * OH * OW * C;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    const long row = i / C;
    const long hw = (long)OH * OW, b = row / hw;
    const int p = (int)(row - b * hw), oy = p / OW, ox = p - oy * OW;
    float best = -3.0e38f;
    int arg = 0;
    for (int t = 0; t < 9; ++t) {
      const int iy = oy * 2 - 1 + t / 3, ix = ox * 2 - 1 + t % 3;
      if (iy < 0 || iy >= H || ix < 0 || ix >= W) continue;
      const float v = bf2f(x[((b * H + iy) * W + ix) * C + c]);
      if (v > best) { best = v; arg = t; }
    }
    y[i] = f2bf(best);
    am[i] = (uint8_t)arg;
  }
}

__global__ void maxpool3_bwd_kernel(const bf16* dy, const uint8_t* am, bf16* dx, int B, int H, int W, int C, int OH,
                                    int OW) {
  const long n = (long)B * H * W * C;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    const long row = i / C;
    const long hw = (long)H * W, b = row / hw;
    const int p = (int)(row - b * hw), iy = p / W, ix = p - iy * W;
    float g = 0.f;
    // outputs whose window (oy*2-1 .. oy*2+1) covers iy
    for (int oy = (iy + 1) / 2 - 1; oy <= (iy + 1) / 2; ++oy) {
      if (oy < 0 || oy >= OH || iy < oy * 2 - 1 || iy > oy * 2 + 1) continue;
      for (int ox = (ix + 1) / 2 - 1; ox <= (ix + 1) / 2; ++ox) {
        if (ox < 0 || ox >= OW || ix < ox * 2 - 1 || ix > ox * 2 + 1) continue;
        const long o = ((b * OH + oy) * OW + ox) * C + c;
        const int t = (iy - (oy * 2 - 1)) * 3 + (ix - (ox * 2 - 1));
        if (am[o] == t) g += bf2f(dy[o]);
      }
    }
    dx[i] = f2bf(g);
  }
}

int ew_grid(long n) {
  long g = (n + 255) / 256;
  if (g > 4096) g = 4096;
  return g < 1 ? 1 : (int)g;
}

}  // namespace

void launch_bn_stats(const BnArgs& a, hipStream_t s) {
  check(a);
  const size_t lds = (size_t)(NT / (a.C / 8)) * 2 * a.C * sizeof(float);
  hipLaunchKernelGGL(bn_stats_kernel, dim3(grid_for(a.R, a.C, 1024, 8)), dim3(NT), lds, s, a);
}

void launch_bn_apply(const BnArgs& a, hipStream_t s) {
  check(a);
  if (a.res && (a.RC % 8 || a.RC > a.C)) throw std::runtime_error("bn_apply: residual channels");
  hipLaunchKernelGGL(bn_apply_kernel, dim3(grid_for(a.R, a.C, 2048, 2)), dim3(NT), 0, s, a);
}

void launch_bn_bwd_stats(const BnArgs& a, hipStream_t s) {
  check(a);
  const size_t lds = (size_t)(NT / (a.C / 8)) * 2 * a.C * sizeof(float);
  hipLaunchKernelGGL(bn_bwd_stats_kernel, dim3(grid_for(a.R, a.C, 1024, 8)), dim3(NT), lds, s, a);
}

void launch_bn_bwd_apply(const BnArgs& a, hipStream_t s) {
  check(a);
  hipLaunchKernelGGL(bn_bwd_apply_kernel, dim3(grid_for(a.R, a.C, 2048, 2)), dim3(NT), 0, s, a);
}

void launch_shortcut_grad_add(const bf16* g, bf16* dx, int B, int OH, int OW, int C, int XH, int XW, int XC,
                              int stride, hipStream_t s) {
  if (XC % 8 || C % 8 || XC > C) throw std::runtime_error("shortcut_grad_add: channels");
  hipLaunchKernelGGL(shortcut_grad_kernel, dim3(ew_grid((long)B * OH * OW * XC / 8)), dim3(256), 0, s, g, dx, B, OH,
                     OW, C, XH, XW, XC, stride);
}

void launch_gap_fwd(const bf16* x, bf16* y, int B, int HW, int C, hipStream_t s) {
  const int t = C / 8;
  if (C % 8 || t > 256 || (t & (t - 1))) throw std::runtime_error("gap: C must be 8 * 2^k <= 2048");
  hipLaunchKernelGGL(gap_fwd_kernel, dim3(B), dim3(256), 0, s, x, y, B, HW, C);
}

void launch_gap_bwd(const bf16* dy, bf16* dx, int B, int HW, int C, hipStream_t s) {
  if (C % 8) throw std::runtime_error("gap: C % 8");
  hipLaunchKernelGGL(gap_bwd_kernel, dim3(ew_grid((long)B * HW * C / 8)), dim3(256), 0, s, dy, dx, B, HW, C);
}

void launch_maxpool3_fwd(const bf16* x, bf16* y, uint8_t* am, int B, int H, int W, int C, int OH, int OW,
                         hipStream_t s) {
  hipLaunchKernelGGL(maxpool3_fwd_kernel, dim3(ew_grid((long)B * OH * OW * C)), dim3(256), 0, s, x, y, am, B, H, W,
                     C, OH, OW);
}

void launch_maxpool3_bwd(const bf16* dy, const uint8_t* am, bf16* dx, int B, int H, int W, int C, int OH, int OW,
                         hipStream_t s) {
  hipLaunchKernelGGL(maxpool3_bwd_kernel, dim3(ew_grid((long)B * H * W * C)), dim3(256), 0, s, dy, am, dx, B, H, W,
                     C, OH, OW);
}

}  // namespace dtfe
