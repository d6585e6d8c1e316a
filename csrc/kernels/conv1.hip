// Single-channel first conv layer (MNIST CNN conv1: 5x5, 1 -> 32, SAME, + ReLU +
// 2x2 max-pool), forward and weight gradient, as dedicated kernels.
//
// With C = 1 the implicit-GEMM K is only 25: the generic loader would spend
// its time on address arithmetic for 8 scalar taps per chunk.  Here each
// workgroup stages whole zero-padded 32x32 images in LDS once; the MFMA
// A fragment (16 output pixels x 32 taps) is read straight from the LDS image
// (tap (kh,kw) of pixel (y,x) = img[y+kh][x+kw]), the 32x32 weight tile is a
// register-resident B fragment, and rows are enumerated by pool window so the
// 4 rows of a lane's accumulator are one 2x2 window (max/argmax in registers).
//
// The weight gradient consumes the POOLED gradient dP (already ReLU-masked by
// its producer) and the argmax: the only non-zero full-resolution gradient of
// window p, channel c sits at argmax[p][c], so
//     dW[c][kh][kw] += dP[p][c] * x[2ph+dy+kh-2][2pw+dx+kw-2],   db[c] += dP[p][c]
// - 25 FMAs per (window, channel) against the LDS image, no full-resolution
// gradient tensor ever written (4x fewer bytes than un-pooling first).
#include "common.h"
#include "conv1.h"

namespace dtfe {

constexpr int IMG = 28, PADW = 32, KS = 5, CO = 32, PO = 14;

// stage N images [28x28] (bf16) into zero-padded [32][32] f32 LDS images.
// A 28-pixel row is 7 chunks of 4 bf16 (8 B, aligned): all loads are issued
// before any LDS write (unrolled, independent) so their latencies overlap.
template <int N>
__device__ __forceinline__ void stage_images(const bf16* x, int b0, int B, float* img) {
  for (int i = threadIdx.x; i < N * PADW * PADW / 4; i += 256)
    reinterpret_cast<f32x4_t*>(img)[i] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  constexpr int CH = N * IMG * 7;  // 8-byte chunks
  constexpr int PER = (CH + 255) / 256;
  u32x2_t v[PER];
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int c = threadIdx.x + j * 256;
    const int im = c / (IMG * 7);
    v[j] = u32x2_t{0u, 0u};
    if (c < CH && b0 + im < B)
      v[j] = *reinterpret_cast<const u32x2_t*>(x + (long)(b0 + im) * IMG * IMG + (c % (IMG * 7)) * 4);
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int c = threadIdx.x + j * 256;
    if (c < CH) {
      const int im = c / (IMG * 7), rc = c % (IMG * 7), r = rc / 7, col = (rc % 7) * 4;
      float* d = img + im * PADW * PADW + (r + 2) * PADW + col + 2;
      d[0] = __uint_as_float(v[j][0] << 16);
      d[1] = __uint_as_float(v[j][0] & 0xffff0000u);
      d[2] = __uint_as_float(v[j][1] << 16);
      d[3] = __uint_as_float(v[j][1] & 0xffff0000u);
    }
  }
}

template <int IMGS>
__global__ __launch_bounds__(256) void conv1_fwd_pool_kernel(Conv1Args a) {
  __shared__ float img[IMGS * PADW * PADW];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int b0 = blockIdx.x * IMGS;
  stage_images<IMGS>(a.x, b0, a.B, img);
  // B fragments: W[co][tap] for co tiles 0..15 / 16..31, taps k = 8*(lane>>4)+j (taps >= 25 are 0)
  bf16x8_t bw[2];
#pragma unroll
  for (int nt = 0; nt < 2; ++nt) {
    s16x8_t v;
    const int co = nt * 16 + (lane & 15);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int tap = 8 * (lane >> 4) + j;
      v[j] = tap < KS * KS ? (short)a.w[co * KS * KS + tap] : (short)0;
    }
    bw[nt] = __builtin_bit_cast(bf16x8_t, v);
  }
  float bias[2];
#pragma unroll
  for (int nt = 0; nt < 2; ++nt) bias[nt] = a.bias ? a.bias[nt * 16 + (lane & 15)] : 0.f;
  // per-lane tap offsets into the padded image for the A fragment
  int toff[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int tap = 8 * (lane >> 4) + j;
    toff[j] = tap < KS * KS ? (tap / KS) * PADW + (tap % KS) : -1;
  }
  __syncthreads();

  constexpr int TILES = PO * PO * 4 / 16;  // 49 tiles of 16 rows (4 windows) per image
  for (int t = wid; t < IMGS * TILES; t += 4) {
    const int im = t / TILES, tile = t % TILES;
    if (b0 + im >= a.B) break;
    // A fragment: row = lane&15 -> window (tile*4 + row/4), quadrant q = row&3
    const int row = lane & 15;
    const int win = tile * 4 + (row >> 2), q = row & 3;
    const int ph = win / PO, pw = win % PO;
    const int y = 2 * ph + (q >> 1), x = 2 * pw + (q & 1);
    const float* base = img + im * PADW * PADW + y * PADW + x;
    s16x8_t av;
#pragma unroll
    for (int j = 0; j < 8; ++j) av[j] = toff[j] >= 0 ? (short)f2bf(base[toff[j]]) : (short)0;
    const bf16x8_t af = __builtin_bit_cast(bf16x8_t, av);
    // each lane's accumulator rows (lane>>4)*4 .. +3 = window tile*4 + (lane>>4)
    const int owin = tile * 4 + (lane >> 4);
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
      f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bw[nt], acc, 0, 0, 0);
      int am = 0;
      float mx = acc[0];
#pragma unroll
      for (int j = 1; j < 4; ++j) if (acc[j] > mx) { mx = acc[j]; am = j; }
      const float v = fmaxf(mx + bias[nt], 0.f);
      const long o = ((long)(b0 + im) * PO * PO + owin) * CO + nt * 16 + (lane & 15);
      a.y[o] = f2bf(v);
      a.argmax[o] = (uint8_t)am;
    }
  }
}

template <int IMGS>
__global__ __launch_bounds__(256) void conv1_wgrad_pooled_kernel(Conv1Args a) {
  __shared__ float img[IMGS * PADW * PADW];
  __shared__ float red[8][CO][KS * KS + 1];
  __shared__ __attribute__((aligned(16))) bf16 gl[IMGS * PO * PO * CO];
  __shared__ __attribute__((aligned(16))) uint8_t al[IMGS * PO * PO * CO];
  const int b0 = blockIdx.x * IMGS;
  const int co = threadIdx.x & 31, pg = threadIdx.x >> 5;  // 8 window groups
  // stage the block's pooled gradient + argmax rows in LDS with 16-byte loads,
  // all issued before the image staging so their latencies overlap
  constexpr int NW = IMGS * PO * PO * CO;               // elements
  constexpr int GCH = NW * 2 / 16, ACH = NW / 16;        // 16-byte chunks
  constexpr int GPER = (GCH + 255) / 256, APER = (ACH + 255) / 256;
  u32x4_t gr[GPER], ar[APER];
  const long e0 = (long)b0 * PO * PO * CO;
  const long ne = (long)min(IMGS, a.B - b0) * PO * PO * CO;
#pragma unroll
  for (int j = 0; j < GPER; ++j) {
    const int c = threadIdx.x + j * 256;
    gr[j] = (c < GCH && c * 8 < ne) ? *reinterpret_cast<const u32x4_t*>(a.dp + e0 + c * 8) : u32x4_t{0u, 0u, 0u, 0u};
  }
#pragma unroll
  for (int j = 0; j < APER; ++j) {
    const int c = threadIdx.x + j * 256;
    ar[j] = (c < ACH && c * 16 < ne) ? *reinterpret_cast<const u32x4_t*>(a.argmax + e0 + c * 16)
                                     : u32x4_t{0u, 0u, 0u, 0u};
  }
  stage_images<IMGS>(a.x, b0, a.B, img);
#pragma unroll
  for (int j = 0; j < GPER; ++j) {
    const int c = threadIdx.x + j * 256;
    if (c < GCH) reinterpret_cast<u32x4_t*>(gl)[c] = gr[j];
  }
#pragma unroll
  for (int j = 0; j < APER; ++j) {
    const int c = threadIdx.x + j * 256;
    if (c < ACH) reinterpret_cast<u32x4_t*>(al)[c] = ar[j];
  }
  __syncthreads();
  float acc[KS * KS + 1];
#pragma unroll
  for (int i = 0; i < KS * KS + 1; ++i) acc[i] = 0.f;
#pragma unroll
  for (int im = 0; im < IMGS; ++im) {
    const float* ib = img + im * PADW * PADW;
    for (int p = pg; p < PO * PO; p += 8) {
      const int o = (im * PO * PO + p) * CO + co;
      const float g = bf2f(gl[o]);
      const int q = al[o];
      const int y = 2 * (p / PO) + (q >> 1), x = 2 * (p % PO) + (q & 1);
      const float* base = ib + (g != 0.f ? y * PADW + x : 0);  // padded coords: tap (kh,kw) at base[kh*32+kw]
#pragma unroll
      for (int kh = 0; kh < KS; ++kh)
#pragma unroll
        for (int kw = 0; kw < KS; ++kw) acc[kh * KS + kw] = fmaf(g, base[kh * PADW + kw], acc[kh * KS + kw]);
      acc[KS * KS] += g;
    }
  }
#pragma unroll
  for (int i = 0; i < KS * KS + 1; ++i) red[pg][co][i] = acc[i];
  __syncthreads();
  for (int i = threadIdx.x; i < CO * (KS * KS + 1); i += 256) {
    const int c = i / (KS * KS + 1), k = i % (KS * KS + 1);
    float s = 0.f;
#pragma unroll
    for (int g = 0; g < 8; ++g) s += red[g][c][k];
    if (k < KS * KS) atomicAdd(a.dw + c * KS * KS + k, s * a.scale);
    else if (a.db) atomicAdd(a.db + c, s * a.scale);
  }
}

void launch_conv1_fwd_pool(const Conv1Args& a, hipStream_t s) {
  constexpr int IMGS = 2;
  hipLaunchKernelGGL(conv1_fwd_pool_kernel<IMGS>, dim3((a.B + IMGS - 1) / IMGS), dim3(256), 0, s, a);
}

void launch_conv1_wgrad_pooled(const Conv1Args& a, hipStream_t s) {
  constexpr int IMGS = 2;
  hipLaunchKernelGGL(conv1_wgrad_pooled_kernel<IMGS>, dim3((a.B + IMGS - 1) / IMGS), dim3(256), 0, s, a);
}

}  // namespace dtfe
