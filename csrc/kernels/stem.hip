// ImageNet stem: 7x7 / stride 2 / pad 3 convolution, 3 -> 64 channels, 224x224 -> 112x112 (NHWC,
// bf16), forward and weight gradient as dedicated kernels (ResNet-50 "conv2d", BASELINE.json
// config 5).  The generic paths cost 1.5 ms (fwd) + 1.8 ms (wgrad) per B=256 step: with C = 3
// the implicit-GEMM K = 147 is one awkward tile and every A fragment gathers 8 scalars.
//
// Layout trick: with stride 2 and C = 3, the 21 values (kw, c) of kernel row kh for output pixel
// ox are 21 CONSECUTIVE elements of the zero-padded input row, starting at element 6*ox.  The
// reduction index is therefore taken as k = kh*24 + kw*3 + c (rows padded 21 -> 24): an MFMA
// k-chunk of 8 is one contiguous, 4-byte aligned run of an LDS row (4 ds_read_b32) and K = 168
// is 6 chunks of 32 (the 7th kh row's last chunk and the 3 pad columns carry zero weights).
//
//   forward   one persistent workgroup per CU, work item = (image, 4 output rows): the 13 input
//             rows it needs are staged in LDS (next item's rows prefetched into registers while
//             this one computes), the weights live in registers as B fragments for the whole
//             kernel (14 waves = 7 pixel tiles x 2 channel halves), the 4 x 112 x 64 output block
//             leaves through an LDS stage as 16-B row-contiguous stores.
//   wgrad     dW[n][k] = sum_pixels dY[p][n] X[p][k]: per work item (image, 2 output rows) the
//             patch matrix X[224 pixels][k] is built in LDS from the staged input rows (11 dword
//             copies per pixel and kh), both operands are read with the gfx950 transposing read
//             ds_read_b64_tr_b16, the accumulators persist across a workgroup's items and are
//             flushed once as register-layout partial slabs; a fixed-order reduce sums the 256
//             slabs (bitwise reproducible, no atomics).
#include <mutex>
#include <stdexcept>

#include "conv.h"
#include "igemm.h"

namespace dtfe {

namespace {

constexpr int SIN = 224, SOUT = 112, SC = 3, SN = 64, SK = 7;
constexpr int ROWE = SIN * SC;        // 672 elements of one input row
constexpr int RW = 704;               // LDS row: 9 zero elements (3 pad pixels) + 672 + zero tail
constexpr int NCH_ROW = ROWE / 8;     // 84 16-B chunks per input row
constexpr int KP = 24;                // k per kernel row, padded (21 -> 24)

// ------------------------------------------------------------------ forward
constexpr int F_RPI = 4;              // output rows per work item
constexpr int F_IR = 2 * F_RPI + 5;   // input rows per item (13)
constexpr int F_T = 896;              // 14 waves
constexpr int F_NPF = (F_IR * NCH_ROW + F_T - 1) / F_T;  // 2

// part (optional): BatchNorm partials of each work item's stored (bf16) output block, the igemm
// epilogue's [items][3][64] layout (K = the block's first pixel, shifted sum, shifted sum of squares)
__global__ __launch_bounds__(F_T) void stem_fwd_kernel(const bf16* __restrict__ x, const bf16* __restrict__ w,
                                                        bf16* __restrict__ y, int B, float* __restrict__ part) {
  __shared__ __attribute__((aligned(16))) bf16 rows[F_IR * RW];
  __shared__ __attribute__((aligned(16))) bf16 ost[F_RPI * SOUT * SN];
  __shared__ float red[F_T / SN][2][SN];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int ct = wid % 7, hf = wid / 7;  // 16-pixel column tile, 32-channel half
  const int g = lane >> 4, i16 = lane & 15;
  for (int i = tid; i < F_IR * RW / 2; i += F_T) reinterpret_cast<uint32_t*>(rows)[i] = 0u;

  // weights as register-resident B fragments: step s, lane k-chunk 4s+g = (kh, sub)
  bf16x8_t bw[2][6];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int s = 0; s < 6; ++s) {
      const int n = (2 * hf + t) * 16 + i16, chunk = 4 * s + g, kh = chunk / 3, sub = chunk - kh * 3;
      s16x8_t v;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int kk = 8 * sub + j;
        v[j] = (chunk < 21 && kk < 21) ? (short)w[n * 147 + kh * 21 + kk] : (short)0;
      }
      bw[t][s] = __builtin_bit_cast(bf16x8_t, v);
    }
  // this lane's A row (output pixel ox) and per-step row / column offsets
  const int ox = 16 * ct + i16;
  int aoff[6];
  bool aok[6];
#pragma unroll
  for (int s = 0; s < 6; ++s) {
    const int chunk = 4 * s + g, kh = chunk / 3, sub = chunk - kh * 3;
    aok[s] = chunk < 21;
    aoff[s] = (aok[s] ? kh : 0) * RW + 6 * ox + 8 * sub;
  }

  const int items = B * (SOUT / F_RPI);
  u32x4_t pf[F_NPF];
  auto load = [&](int it) {
    const int b = it / (SOUT / F_RPI), iy0 = (it % (SOUT / F_RPI)) * 2 * F_RPI - 3;
#pragma unroll
    for (int j = 0; j < F_NPF; ++j) {
      const int c = tid + j * F_T;
      pf[j] = u32x4_t{0u, 0u, 0u, 0u};
      if (c < F_IR * NCH_ROW) {
        const int r = c / NCH_ROW, cc = c - r * NCH_ROW, iy = iy0 + r;
        if ((unsigned)iy < (unsigned)SIN)
          pf[j] = *reinterpret_cast<const u32x4_t*>(x + ((long)b * SIN + iy) * ROWE + cc * 8);
      }
    }
  };
  auto put = [&]() {  // interior starts at element 9 (odd): 2-byte stores
#pragma unroll
    for (int j = 0; j < F_NPF; ++j) {
      const int c = tid + j * F_T;
      if (c < F_IR * NCH_ROW) {
        const int r = c / NCH_ROW, cc = c - r * NCH_ROW;
        bf16* d = rows + r * RW + 9 + cc * 8;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          d[2 * e] = (bf16)(pf[j][e] & 0xffffu);
          d[2 * e + 1] = (bf16)(pf[j][e] >> 16);
        }
      }
    }
  };

  int it = blockIdx.x;
  if (it < items) load(it);
  __syncthreads();  // zero pads before the first interior write
  for (; it < items; it += gridDim.x) {
    put();
    __syncthreads();
    if (it + (int)gridDim.x < items) load(it + gridDim.x);
    // one output row at a time (8 accumulator registers; the 14-wave workgroup allows 128 VGPRs),
    // staged as [4 rows][112][64] (lane: pixels 16ct + 4g + j, channel (2hf + t)*16 + i16)
#pragma unroll
    for (int d = 0; d < F_RPI; ++d) {
      f32x4_t acc[2] = {f32x4_t{0.f, 0.f, 0.f, 0.f}, f32x4_t{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
      for (int s = 0; s < 6; ++s) {
        const uint32_t* p = reinterpret_cast<const uint32_t*>(rows + 2 * d * RW + aoff[s]);
        u32x4_t v = {p[0], p[1], p[2], p[3]};
        if (!aok[s]) v = u32x4_t{0u, 0u, 0u, 0u};
        const bf16x8_t af = __builtin_bit_cast(bf16x8_t, v);
        acc[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bw[0][s], acc[0], 0, 0, 0);
        acc[1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bw[1][s], acc[1], 0, 0, 0);
      }
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          ost[(d * SOUT + 16 * ct + 4 * g + j) * SN + (2 * hf + t) * 16 + i16] = f2bf(acc[t][j]);
    }
    __syncthreads();
    const long base = ((long)(it / (SOUT / F_RPI)) * SOUT + (it % (SOUT / F_RPI)) * F_RPI) * SOUT * SN;
    for (int c = tid; c < F_RPI * SOUT * SN / 8; c += F_T)
      *reinterpret_cast<u32x4_t*>(y + base + c * 8) = *reinterpret_cast<const u32x4_t*>(ost + c * 8);
    if (part) {
      // thread (channel c, row group rg) sums pixels rg, rg + 14, ... around the block's first
      // pixel; the 14 row groups are folded in order (deterministic)
      constexpr int RG = F_T / SN, NPIX = F_RPI * SOUT;
      const int c = tid % SN, rg = tid / SN;
      const float k = bf2f(ost[c]);
      float sm = 0.f, sq = 0.f;
      for (int p = rg; p < NPIX; p += RG) {
        const float d = bf2f(ost[p * SN + c]) - k;
        sm += d;
        sq += d * d;
      }
      red[rg][0][c] = sm;
      red[rg][1][c] = sq;
      __syncthreads();
      if (tid < SN) {
        float S = 0.f, Q = 0.f;
        for (int r = 0; r < RG; ++r) {
          S += red[r][0][tid];
          Q += red[r][1][tid];
        }
        float* pp = part + (long)it * 3 * SN + tid;
        pp[0] = k;
        pp[SN] = S;
        pp[2 * SN] = Q;
      }
    }
  }
}

// ------------------------------------------------------------------ weight gradient
constexpr int W_RPI = 2;                     // output rows per work item
constexpr int W_IR = 2 * W_RPI + 5;          // 9 input rows
constexpr int W_PIX = W_RPI * SOUT;          // 224 pixels = 7 k-steps of 32
constexpr int W_T = 512;                     // 8 waves: 2 channel pairs x 4 column groups
constexpr int XP = 176;                      // patch-matrix pitch (11 x 16 elements: odd multiple of 16)
constexpr int DP = 80;                       // dY pixel pitch (odd multiple of 16 >= 64)
constexpr int W_CT = XP / 16;                // 11 column tiles
constexpr int W_NPFX = (W_IR * NCH_ROW + W_T - 1) / W_T;  // 2
constexpr int W_NPFD = (W_PIX * SN / 8 + W_T - 1) / W_T;  // 4
constexpr int W_SLAB = 8 * 2 * 3 * 64 * 4;   // floats of one workgroup's register-layout partial

__global__ __launch_bounds__(W_T) void stem_wgrad_kernel(const bf16* __restrict__ x, const bf16* __restrict__ dy,
                                                          float* __restrict__ part, int B) {
  extern __shared__ __attribute__((aligned(16))) bf16 lds[];
  bf16* rows = lds;                       // [9][RW]
  bf16* xc = rows + W_IR * RW;            // [224][XP]
  bf16* dimg = xc + W_PIX * XP;           // [224][DP]
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int mp = wid & 1, cg = wid >> 1;  // channels 32*mp .. +32, column tiles cg, cg+4, cg+8
  const int g = lane >> 4, i16 = lane & 15, q = i16 >> 2, p4 = i16 & 3;
  for (int i = tid; i < (W_IR * RW + W_PIX * XP) / 2; i += W_T) reinterpret_cast<uint32_t*>(lds)[i] = 0u;

  // transposed-read offsets (k = pixel): lane (g, q, p4) of read h covers pixel 16h + 4g + q
  int doff[2], koff[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int kl = 16 * h + 4 * g + q;
    doff[h] = kl * DP + 4 * p4;
    koff[h] = kl * XP + 4 * p4;
  }
  f32x4_t acc[2][3];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int items = B * (SOUT / W_RPI);
  u32x4_t px[W_NPFX], pd[W_NPFD];
  auto load = [&](int it) {
    const int b = it / (SOUT / W_RPI), oy0 = (it % (SOUT / W_RPI)) * W_RPI, iy0 = 2 * oy0 - 3;
#pragma unroll
    for (int j = 0; j < W_NPFX; ++j) {
      const int c = tid + j * W_T;
      px[j] = u32x4_t{0u, 0u, 0u, 0u};
      if (c < W_IR * NCH_ROW) {
        const int r = c / NCH_ROW, cc = c - r * NCH_ROW, iy = iy0 + r;
        if ((unsigned)iy < (unsigned)SIN)
          px[j] = *reinterpret_cast<const u32x4_t*>(x + ((long)b * SIN + iy) * ROWE + cc * 8);
      }
    }
    const bf16* dsrc = dy + ((long)b * SOUT + oy0) * SOUT * SN;  // 2 rows x 112 x 64, contiguous
#pragma unroll
    for (int j = 0; j < W_NPFD; ++j) {
      const int c = tid + j * W_T;
      if (c < W_PIX * SN / 8) pd[j] = *reinterpret_cast<const u32x4_t*>(dsrc + c * 8);
    }
  };
  auto put = [&]() {
#pragma unroll
    for (int j = 0; j < W_NPFX; ++j) {
      const int c = tid + j * W_T;
      if (c < W_IR * NCH_ROW) {
        const int r = c / NCH_ROW, cc = c - r * NCH_ROW;
        bf16* d = rows + r * RW + 9 + cc * 8;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          d[2 * e] = (bf16)(px[j][e] & 0xffffu);
          d[2 * e + 1] = (bf16)(px[j][e] >> 16);
        }
      }
    }
#pragma unroll
    for (int j = 0; j < W_NPFD; ++j) {
      const int c = tid + j * W_T;
      if (c < W_PIX * SN / 8) {
        const int p = c >> 3, cc = c & 7;
        *reinterpret_cast<u32x4_t*>(dimg + p * DP + cc * 8) = pd[j];
      }
    }
  };

  int it = blockIdx.x;
  if (it < items) load(it);
  __syncthreads();
  for (; it < items; it += gridDim.x) {
    put();
    __syncthreads();
    if (it + (int)gridDim.x < items) load(it + gridDim.x);
    // patch matrix: xc[p][kh*24 + kw*3 + c] = 11 dwords from row 2d + kh at element 6*ox
    // (dword 10 carries one element of the next pixel into the pad column kh*24 + 21: its dW
    // column is never flushed)
    for (int i = tid; i < W_PIX * SK * 11; i += W_T) {
      const int p = i / (SK * 11), rem = i - p * (SK * 11), kh = rem / 11, wd = rem - kh * 11;
      const int d = p >= SOUT, oxp = p - d * SOUT;
      reinterpret_cast<uint32_t*>(xc + p * XP + kh * KP)[wd] =
          reinterpret_cast<const uint32_t*>(rows + (2 * d + kh) * RW + 6 * oxp)[wd];
    }
    __syncthreads();
#pragma unroll
    for (int s = 0; s < W_PIX / 32; ++s) {
      bf16x8_t af[2];
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        const bf16* base = dimg + s * 32 * DP + (2 * mp + m) * 16;
        const s16x4_t h0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4_t, base + doff[0]));
        const s16x4_t h1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4_t, base + doff[1]));
        const s16x8_t v = {h0[0], h0[1], h0[2], h0[3], h1[0], h1[1], h1[2], h1[3]};
        af[m] = __builtin_bit_cast(bf16x8_t, v);
      }
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const int ctile = cg + 4 * c;
        if (ctile >= W_CT) break;  // wave-uniform
        const bf16* base = xc + s * 32 * XP + ctile * 16;
        const s16x4_t h0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4_t, base + koff[0]));
        const s16x4_t h1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4_t, base + koff[1]));
        const s16x8_t v = {h0[0], h0[1], h0[2], h0[3], h1[0], h1[1], h1[2], h1[3]};
        const bf16x8_t bfr = __builtin_bit_cast(bf16x8_t, v);
#pragma unroll
        for (int m = 0; m < 2; ++m) acc[m][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[m], bfr, acc[m][c], 0, 0, 0);
      }
    }
    __syncthreads();  // rows / xc / dimg are rewritten by the next item
  }
  // register-layout partial slab [wave][m][c][lane] of f32x4
  f32x4_t* pv = reinterpret_cast<f32x4_t*>(part + (long)blockIdx.x * W_SLAB) + (long)wid * 6 * 64 + lane;
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int c = 0; c < 3; ++c) pv[(m * 3 + c) * 64] = acc[m][c];
}

// dw[n][kh][kw][c] (+)= scale * sum over the nblk slabs, fixed order (16 strided subsets, then
// the subsets in order through LDS)
__global__ __launch_bounds__(256) void stem_wgrad_reduce_kernel(const float* __restrict__ part, int nblk, float* dw,
                                                                float scale, int accumulate) {
  __shared__ f32x4_t red[16][17];
  const int c16 = threadIdx.x & 15, pg = threadIdx.x >> 4;
  const int v = blockIdx.x * 16 + c16;  // f32x4 index within a slab
  f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
  if (v < W_SLAB / 4)
    for (int p = pg; p < nblk; p += 16) acc += *reinterpret_cast<const f32x4_t*>(part + (long)p * W_SLAB + 4 * v);
  red[pg][c16] = acc;
  __syncthreads();
  if (pg != 0 || v >= W_SLAB / 4) return;
  f32x4_t t = red[0][c16];
#pragma unroll
  for (int k = 1; k < 16; ++k) t += red[k][c16];
  const int lane = v & 63, r = v >> 6, c = r % 3, m = (r / 3) & 1, wv = r / 6;
  const int mp = wv & 1, cg = wv >> 1, ctile = cg + 4 * c;
  if (ctile >= W_CT) return;
  const int col = ctile * 16 + (lane & 15), kh = col / KP, kk = col - kh * KP;
  if (kh >= SK || kk >= 21) return;
  const int n0 = (2 * mp + m) * 16 + (lane >> 4) * 4;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    float* d = dw + (long)(n0 + j) * 147 + kh * 21 + kk;
    *d = (accumulate ? *d : 0.f) + scale * t[j];
  }
}

bool stem_shape(const ConvGeom& g) {
  return g.C == SC && g.KH == SK && g.KW == SK && g.stride == 2 && g.pad == 3 && g.H == SIN && g.W == SIN &&
         g.OH == SOUT && g.OW == SOUT && g.Cout == SN && !g.pool_order;
}

std::mutex g_mu;
struct Scratch {
  float* ws = nullptr;
  size_t bytes = 0;
};
Scratch g_ws[64];

float* stem_workspace(size_t bytes, hipStream_t s) {
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::lock_guard<std::mutex> lk(g_mu);
  Scratch& d = g_ws[dev];
  if (d.bytes < bytes) {
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    (void)hipStreamIsCapturing(s, &st);
    if (st != hipStreamCaptureStatusNone)
      throw std::runtime_error("stem wgrad: workspace growth inside a graph capture (run the step eagerly first)");
    if (d.ws) {
      (void)hipStreamSynchronize(s);
      (void)hipFree(d.ws);
    }
    if (hipMalloc(&d.ws, bytes) != hipSuccess) throw std::runtime_error("stem wgrad: workspace alloc");
    d.bytes = bytes;
  }
  return d.ws;
}

}  // namespace

bool launch_stem_fwd(const ConvFwdArgs& a, hipStream_t s, bool* stats_done) {
  if (!stem_shape(a.g) || a.bias || a.act != ACT_NONE || a.argmax) return false;
  const int items = a.g.B * (SOUT / F_RPI);
  const int grid = items < 256 ? items : 256;
  // BatchNorm statistics from the epilogue's per-block partials (2 small fold launches instead of
  // a 411 MB re-read of y at B = 256)
  float* part = a.bn_stats ? bn_part_buffer(items, SN, s) : nullptr;
  hipLaunchKernelGGL(stem_fwd_kernel, dim3(grid), dim3(F_T), 0, s, a.x, a.w, a.y, a.g.B, part);
  if (part) launch_bn_part_reduce(part, items, SN, (long)a.g.B * SOUT * SOUT, F_RPI * SOUT, a.bn_stats, s);
  if (stats_done) *stats_done = part != nullptr;
  return true;
}

bool launch_stem_wgrad(const ConvWgradArgs& a, hipStream_t s, bool accumulate) {
  if (!stem_shape(a.g) || a.db) return false;
  const int items = a.g.B * (SOUT / W_RPI);
  const int grid = items < 256 ? items : 256;
  float* part = stem_workspace((size_t)grid * W_SLAB * sizeof(float), s);
  const size_t lds = (size_t)(W_IR * RW + W_PIX * XP + W_PIX * DP) * sizeof(bf16);
  (void)hipFuncSetAttribute((const void*)stem_wgrad_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(stem_wgrad_kernel, dim3(grid), dim3(W_T), lds, s, a.x, a.dz, part, a.g.B);
  hipLaunchKernelGGL(stem_wgrad_reduce_kernel, dim3((W_SLAB / 4 + 15) / 16), dim3(256), 0, s, part, grid, a.dw,
                     a.scale, accumulate ? 1 : 0);
  return true;
}

}  // namespace dtfe
