// Whole-image LDS convolutions for small feature maps - see imgconv.h.
//
// Why: an implicit GEMM over im2col re-reads every input pixel KH*KW times
// from L2/MALL (the MNIST conv2 A operand is 25x its 12.8 MB input per step);
// at these image sizes a whole padded image (<= 41 KB) fits in LDS, so each
// workgroup loads its image exactly once and every A fragment is one
// ds_read_b128 (8 channels of one pixel+tap).  Rows are output pixels of the
// image (pool-window order when the 2x2 max-pool is fused), so the epilogue
// pools the 4 rows each lane holds in registers.
//
// Weight gradient: both operands come from LDS images through the gfx950
// transposing read ds_read_b64_tr_b16: the reduction index k is the output
// pixel (enumerated over power-of-two-wide rows, so 4 consecutive k are 4
// consecutive pixels of one row and a k-step of 32 advances by whole rows),
// A = dY image [pixel][n], B = source image at pixel+tap.
//
// rocprof PMC of the first version showed 13-20 VALU per MFMA (integer
// divisions for the tap decode every k-step); the k loops below carry all
// addresses incrementally, so the inner loop is loads + MFMAs.
#include "imgconv.h"

#include <stdexcept>

namespace dtfe {

constexpr int IC_THREADS = 256;

__device__ __forceinline__ int fdiv(int m, int d, float inv_d) {  // exact m / d for 0 <= m < 2^22
  int q = (int)((float)m * inv_d);
  const int r = m - q * d;
  return q + (r >= d) - (r < 0);
}

// ------------------------------------------------------------------ staging
// LDS image [LH][LW][CS] (CS a multiple of 8) with source pixel (sy, sx) at
// (sy + lo, sx + lo); zero elsewhere.
// With src_pooled the source is un-pooled on the fly:
//   value(sy, sx, c) = argmax[sy/2][sx/2][c] == (sy&1)*2+(sx&1) ? pooled[sy/2][sx/2][c] : 0.
// Then `extra` more zero elements follow the image (slack for dummy reads).
__device__ __forceinline__ void stage_image(bf16* img, int LH, int LW, int lo, int SH, int SW, int CS,
                                            const bf16* src, const bf16* src_pooled, const uint8_t* src_argmax,
                                            long b, int extra) {
  const int cpp = CS >> 3;             // 16-byte chunks per pixel (1, 2, 4, 8)
  const int ppi = IC_THREADS / cpp;    // pixels per pass
  const int cq = threadIdx.x % cpp, ch = cq * 8;
  const int npix = LH * LW;
  const float inv_lw = 1.f / (float)LW;
  for (int p0 = threadIdx.x / cpp; p0 < npix; p0 += ppi * 4) {
    u32x4_t v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int pix = p0 + u * ppi;
      v[u] = u32x4_t{0u, 0u, 0u, 0u};
      if (pix < npix) {
        const int ly = fdiv(pix, LW, inv_lw), sy = ly - lo, sx = pix - ly * LW - lo;
        if (sy >= 0 && sy < SH && sx >= 0 && sx < SW) {
          if (src) {
            v[u] = *reinterpret_cast<const u32x4_t*>(src + ((b * SH + sy) * SW + sx) * CS + ch);
          } else {
            const long po = ((b * (SH >> 1) + (sy >> 1)) * (SW >> 1) + (sx >> 1)) * CS + ch;
            const u32x4_t pv = *reinterpret_cast<const u32x4_t*>(src_pooled + po);
            const u32x2_t am = *reinterpret_cast<const u32x2_t*>(src_argmax + po);
            const uint32_t q = (uint32_t)(((sy & 1) << 1) | (sx & 1));
            // byte e of am == q  -> keep bf16 element e
            uint32_t keep[2];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              const uint32_t x = am[h] ^ (q * 0x01010101u);  // zero bytes where argmax == q
              keep[h] = x;
            }
#pragma unroll
            for (int w = 0; w < 4; ++w) {
              const uint32_t x = keep[w >> 1] >> (16 * (w & 1));
              const uint32_t lo_ok = (x & 0xffu) == 0u ? 0x0000ffffu : 0u;
              const uint32_t hi_ok = (x & 0xff00u) == 0u ? 0xffff0000u : 0u;
              v[u][w] = pv[w] & (lo_ok | hi_ok);
            }
          }
        }
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int pix = p0 + u * ppi;
      if (pix < npix) reinterpret_cast<u32x4_t*>(img)[pix * cpp + cq] = v[u];
    }
  }
  for (int i = threadIdx.x; i < extra / 8; i += IC_THREADS)
    reinterpret_cast<u32x4_t*>(img + (size_t)npix * CS)[i] = u32x4_t{0u, 0u, 0u, 0u};
}

// Few-channel LDS image [LH][LW][CS] (CS <= 4; source [SH][SW][CS] at offset lo), then `extra` zeros.
// The source image is contiguous: its 16-B chunks are loaded up front (all in flight at once), the
// LDS image is zeroed meanwhile, and the chunks' elements are scattered into the padded layout.  (The
// per-element 2-byte global loads before - one dependent round trip per element and channel - held
// ResNet-20's stem at ~25 us per launch, profiles/r5_resnet20_b256_kernels.txt.)  Contains a barrier.
__device__ __forceinline__ void stage_image_small(bf16* img, int LH, int LW, int CS, int lo, int SH, int SW,
                                                  const bf16* src, int extra) {
  const int npix = LH * LW, n = SH * SW * CS;
  const bool vec = (reinterpret_cast<uintptr_t>(src) & 15) == 0;
  const int nch = vec ? n >> 3 : 0;
  constexpr int PF = 4;
  const float inv_cs = 1.f / (float)CS, inv_sw = 1.f / (float)SW;
  auto put = [&](int q, bf16 v) {
    const int p = fdiv(q, CS, inv_cs), c = q - p * CS, sy = fdiv(p, SW, inv_sw), sx = p - sy * SW;
    img[((sy + lo) * LW + sx + lo) * CS + c] = v;
  };
  for (int base = 0; base < nch || base == 0; base += PF * IC_THREADS) {
    u32x4_t v[PF];
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      const int i = base + threadIdx.x + u * IC_THREADS;
      if (i < nch) v[u] = *reinterpret_cast<const u32x4_t*>(src + (long)i * 8);
    }
    if (base == 0) {
      for (int i = threadIdx.x; i < npix * CS + extra; i += IC_THREADS) img[i] = (bf16)0;
      __syncthreads();
    }
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      const int i = base + threadIdx.x + u * IC_THREADS;
      if (i < nch) {
#pragma unroll
        for (int e = 0; e < 8; ++e) put(i * 8 + e, (bf16)((v[u][e >> 1] >> (16 * (e & 1))) & 0xffffu));
      }
    }
    if (nch == 0) break;
  }
  for (int q = nch * 8 + threadIdx.x; q < n; q += IC_THREADS) put(q, src[q]);  // tail / unaligned source
}

// epilogue: lane holds rows (lane>>4)*4 + j of each 16-row tile, column lane&15 of each n-tile
template <int NT, int RT>
__device__ __forceinline__ void imgconv_epilogue(const ImgConvArgs& a, const f32x4_t (&acc)[RT][NT], int t0, int tiles,
                                                 int M, long b, int lane) {
#pragma unroll
  for (int r = 0; r < RT; ++r) {
    const int tile = t0 + 4 * r;
    if (tile >= tiles) break;
    const int m0 = tile * 16 + (lane >> 4) * 4;
#pragma unroll
    for (int n = 0; n < NT; ++n) {
      const int col = n * 16 + (lane & 15);
      if (col >= a.N) continue;
      const float bias = a.bias ? a.bias[col] : 0.f;
      const f32x4_t v = acc[r][n];
      if (a.pool) {
        if (m0 >= M) continue;
        int am = 0;
        float mx = v[0];
#pragma unroll
        for (int j = 1; j < 4; ++j) if (v[j] > mx) { mx = v[j]; am = j; }
        const long o = (b * (M >> 2) + (m0 >> 2)) * a.N + col;
        a.y[o] = f2bf(apply_act(mx + bias, a.act));
        if (a.argmax) a.argmax[o] = (uint8_t)am;
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if (m0 + j >= M) continue;
          const long o = (b * M + m0 + j) * a.N + col;
          float x = apply_act(v[j] + bias, a.act);
          if (a.relu_mask && !(bf2f(a.relu_mask[o]) > 0.f)) x = 0.f;
          a.y[o] = f2bf(x);
        }
      }
    }
  }
}

// -------------------------------------------------------------- fwd / dgrad
template <int NT, int RT>
__global__ __launch_bounds__(IC_THREADS) void imgconv_kernel(ImgConvArgs a) {
  extern __shared__ __attribute__((aligned(16))) bf16 img[];
  const long b = blockIdx.x;
  const int LH = (a.OH - 1) * a.stride + a.KH, LW = (a.OW - 1) * a.stride + a.KW;
  stage_image(img, LH, LW, a.pad, a.SH, a.SW, a.CS, a.src, a.src_pooled, a.src_argmax, b, 0);
  __syncthreads();

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, g = lane >> 4;
  const int M = a.OH * a.OW, tiles = (M + 15) >> 4;
  const int T = a.KH * a.KW, K = T * a.CS, nk = (K + 31) >> 5;
  const int POW = a.OW >> 1;
  // per-lane k-walk start: k = 8g -> (tap, cs); the walk advances 32 per step
  const int tap0 = (8 * g) / a.CS, cs0 = 8 * g - tap0 * a.CS;
  const int kh0 = tap0 / a.KW, kw0 = tap0 - kh0 * a.KW;
  const int row_jump = (LW - a.KW) * a.CS;  // extra LDS offset when kw wraps to the next kernel row
  for (int t0 = wid; t0 < tiles; t0 += 4 * RT) {
    int pix[RT];
#pragma unroll
    for (int r = 0; r < RT; ++r) {
      const int m = (t0 + 4 * r) * 16 + (lane & 15);
      pix[r] = -1;
      if (t0 + 4 * r < tiles && m < M) {
        int oy, ox;
        if (a.pool) {
          const int q = m & 3, w = m >> 2;
          oy = 2 * (w / POW) + (q >> 1);
          ox = 2 * (w % POW) + (q & 1);
        } else {
          oy = m / a.OW;
          ox = m % a.OW;
        }
        pix[r] = (oy * a.stride * LW + ox * a.stride) * a.CS;
      }
    }
    f32x4_t acc[RT][NT];
#pragma unroll
    for (int r = 0; r < RT; ++r)
#pragma unroll
      for (int n = 0; n < NT; ++n) acc[r][n] = f32x4_t{0.f, 0.f, 0.f, 0.f};

    // incremental k walk state (this lane's 8 k values within the 32-wide step)
    int cs = cs0, kw = kw0, kh = kh0;
    int toff = (kh0 * LW + kw0) * a.CS + cs0;                                 // LDS tap offset
    long woff = (long)(a.flip_taps ? (T - 1 - tap0) : tap0) * a.CS + cs0;     // weight k offset
    const bf16* wrow[NT];
    bool colok[NT];
#pragma unroll
    for (int n = 0; n < NT; ++n) {
      const int col = n * 16 + (lane & 15);
      colok[n] = col < a.N;
      wrow[n] = a.w + (long)(colok[n] ? col : 0) * K;
    }
    u32x4_t bcur[NT];
#pragma unroll
    for (int n = 0; n < NT; ++n)
      bcur[n] = (colok[n] && 8 * g < K) ? *reinterpret_cast<const u32x4_t*>(wrow[n] + woff) : u32x4_t{0u, 0u, 0u, 0u};
    for (int s = 0; s < nk; ++s) {
      const bool kv = s * 32 + 8 * g < K;
      const int toff_s = toff;
      // advance the walk to step s+1 and prefetch its weight fragments
      cs += 32;
      toff += 32;
      woff += 32;
      while (cs >= a.CS) {
        cs -= a.CS;
        if (a.flip_taps) woff -= 2 * a.CS;
        if (++kw == a.KW) { kw = 0; ++kh; toff += row_jump; }
      }
      u32x4_t bnext[NT];
      const bool kv1 = (s + 1) * 32 + 8 * g < K;
#pragma unroll
      for (int n = 0; n < NT; ++n)
        bnext[n] = (colok[n] && kv1) ? *reinterpret_cast<const u32x4_t*>(wrow[n] + woff) : u32x4_t{0u, 0u, 0u, 0u};
      bf16x8_t bf[NT];
#pragma unroll
      for (int n = 0; n < NT; ++n) bf[n] = __builtin_bit_cast(bf16x8_t, bcur[n]);
#pragma unroll
      for (int r = 0; r < RT; ++r) {
        u32x4_t v = {0u, 0u, 0u, 0u};
        if (kv && pix[r] >= 0) v = *reinterpret_cast<const u32x4_t*>(img + pix[r] + toff_s);
        const bf16x8_t af = __builtin_bit_cast(bf16x8_t, v);
#pragma unroll
        for (int n = 0; n < NT; ++n) acc[r][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bf[n], acc[r][n], 0, 0, 0);
      }
#pragma unroll
      for (int n = 0; n < NT; ++n) bcur[n] = bnext[n];
    }
    imgconv_epilogue<NT, RT>(a, acc, t0, tiles, M, b, lane);
  }
}

// Few-channel source (network inputs: MNIST 1, CIFAR/ImageNet 3 channels):
// k = tap*CS + c (KH*KW*CS <= 32, one k-step), A fragment = 8 (tap, c) values
// of one output pixel gathered from the LDS image with per-lane constant
// offsets, weights [N][T*CS] held in registers.
// STAGE: the (un-pooled, unmasked) output staged in LDS after the image and stored as 16-B rows
template <int NT, int RT, bool STAGE = false>
__global__ __launch_bounds__(IC_THREADS) void imgconv1_kernel(ImgConvArgs a) {
  extern __shared__ __attribute__((aligned(16))) bf16 img[];
  const long b = blockIdx.x;
  const int LH = (a.OH - 1) * a.stride + a.KH, LW = (a.OW - 1) * a.stride + a.KW;
  const int CS = a.CS;
  bf16* sy = img + (LH * LW * CS + 7) / 8 * 8;
  stage_image_small(img, LH, LW, CS, a.pad, a.SH, a.SW, a.src + b * a.SH * a.SW * CS, 0);
  __syncthreads();
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, g = lane >> 4;
  const int M = a.OH * a.OW, tiles = (M + 15) >> 4, K = a.KH * a.KW * CS, POW = a.OW >> 1;
  int toff[8];
  bf16x8_t bf[NT];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int k = 8 * g + j, tap = k / CS, c = k - tap * CS, kh = tap / a.KW;
    toff[j] = k < K ? (kh * LW + (tap - kh * a.KW)) * CS + c : -1;
  }
#pragma unroll
  for (int n = 0; n < NT; ++n) {
    const int col = n * 16 + (lane & 15);
    s16x8_t v;  // bf16 bit patterns (bf16 is the uint16 storage type: never convert numerically)
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (short)((col < a.N && toff[j] >= 0) ? a.w[(long)col * K + 8 * g + j] : 0);
    bf[n] = __builtin_bit_cast(bf16x8_t, v);
  }
  for (int t0 = wid; t0 < tiles; t0 += 4 * RT) {
    f32x4_t acc[RT][NT];
#pragma unroll
    for (int r = 0; r < RT; ++r) {
      const int m = (t0 + 4 * r) * 16 + (lane & 15);
      int pix = 0;  // rows past M compute garbage that the epilogue drops
      if (t0 + 4 * r < tiles && m < M) {
        int oy, ox;
        if (a.pool) {
          const int q = m & 3, w = m >> 2;
          oy = 2 * (w / POW) + (q >> 1);
          ox = 2 * (w % POW) + (q & 1);
        } else {
          oy = m / a.OW;
          ox = m % a.OW;
        }
        pix = (oy * a.stride * LW + ox * a.stride) * CS;
      }
      s16x8_t av;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const bf16 v = img[pix + (toff[j] < 0 ? 0 : toff[j])];
        av[j] = (short)(toff[j] < 0 ? 0 : v);
      }
      const bf16x8_t af = __builtin_bit_cast(bf16x8_t, av);
#pragma unroll
      for (int n = 0; n < NT; ++n)
        acc[r][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bf[n], f32x4_t{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
    }
    if constexpr (STAGE) {
#pragma unroll
      for (int r = 0; r < RT; ++r) {
        const int tile = t0 + 4 * r;
        if (tile >= tiles) break;
        const int m0 = tile * 16 + (lane >> 4) * 4;
#pragma unroll
        for (int n = 0; n < NT; ++n) {
          const int col = n * 16 + (lane & 15);
          if (col >= a.N) continue;
          const float bias = a.bias ? a.bias[col] : 0.f;
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (m0 + j < M) sy[(m0 + j) * a.N + col] = f2bf(apply_act(acc[r][n][j] + bias, a.act));
        }
      }
    } else {
      imgconv_epilogue<NT, RT>(a, acc, t0, tiles, M, b, lane);
    }
  }
  if constexpr (STAGE) {  // the image's output leaves as contiguous 16-B chunks
    __syncthreads();
    const long ob = b * (long)M * a.N;
    for (int i = threadIdx.x; i < M * a.N / 8; i += IC_THREADS)
      *reinterpret_cast<u32x4_t*>(a.y + ob + i * 8) = *reinterpret_cast<const u32x4_t*>(sy + i * 8);
  }
}

bool imgconv_supported(int SH, int SW, int CS, int N, int KH, int KW, int stride, int pad) {
  const int OH = (SH + 2 * pad - KH) / stride + 1, OW = (SW + 2 * pad - KW) / stride + 1;
  const long LH = (long)(OH - 1) * stride + KH, LW = (long)(OW - 1) * stride + KW;
  if (CS <= 4) return KH * KW * CS <= 32 && N <= 64 && LH * LW * CS * 2 <= 150 * 1024;
  return CS % 8 == 0 && N <= 64 && LH * LW * CS * 2 <= 150 * 1024;
}

template <int NT>
static void launch_nt(const ImgConvArgs& a, size_t lds, hipStream_t s) {
  constexpr int RT = 4;
  if (a.CS <= 4 && !a.pool && !a.relu_mask && a.N % 8 == 0 && !(diag_bits("ic1") & 1)) {
    // few-channel forward (ResNet-20 stem): output staged in LDS, 16-B stores
    const size_t st = (lds + 15) / 16 * 16 + (size_t)a.OH * a.OW * a.N * sizeof(bf16);
    if (st <= 150 * 1024) {
      auto k = imgconv1_kernel<NT, RT, true>;
      if (st > 64 * 1024) (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)st);
      hipLaunchKernelGGL(k, dim3(a.B), dim3(IC_THREADS), st, s, a);
      return;
    }
  }
  auto k = a.CS <= 4 ? imgconv1_kernel<NT, RT> : imgconv_kernel<NT, RT>;
  if (lds > 64 * 1024) (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(k, dim3(a.B), dim3(IC_THREADS), lds, s, a);
}

bool launch_imgconv(const ImgConvArgs& a, hipStream_t s) {
  if (!imgconv_supported(a.SH, a.SW, a.CS, a.N, a.KH, a.KW, a.stride, a.pad))
    throw std::runtime_error("imgconv: shape not supported");
  if (a.CS <= 4 && (!a.src || a.flip_taps || a.dil > 1))
    throw std::runtime_error("imgconv: the few-channel path is forward-only");
  if (a.pool && ((a.OH | a.OW) & 1)) throw std::runtime_error("imgconv: pool needs even output dims");
  if (a.bns.stats && (a.CS <= 4 || !a.src)) throw std::runtime_error("imgconv: BN-on-load needs a plain source");
  if (a.CS <= 4 && launch_conv1_copies_fwd(a, s)) return false;
  bool sc_done = false;
  if (a.CS > 4 && launch_imgconv_persistent(a, s, &sc_done)) return sc_done;
  if (a.bns.stats) throw std::runtime_error("imgconv: BN-on-load needs the persistent kernel (B >= 64)");
  if (a.dil > 1) throw std::runtime_error("imgconv: dilated sources need the persistent kernel (B >= 64)");
  const int LH = (a.OH - 1) * a.stride + a.KH, LW = (a.OW - 1) * a.stride + a.KW;
  const size_t lds = (size_t)LH * LW * a.CS * sizeof(bf16);
  if (a.N <= 16) launch_nt<1>(a, lds, s);
  else if (a.N <= 32) launch_nt<2>(a, lds, s);
  else launch_nt<4>(a, lds, s);
  return false;
}

// ------------------------------------------------------------------- wgrad
// Reduction index k = output pixel oy*OWP + ox, OWP = next power of two >= OW
// (<= 32, so a 32-wide k-step covers whole rows); dummy pixels carry zero dY.
//   A(m = n_out, k = pixel)    = dY[pixel][n]                  (tr read of the dY image)
//   B(n = (tap, c), k = pixel) = src[pixel*stride - pad + tap][c] (tr read of the source image)
// Block = (image group, slab of column tiles); each wave owns CT column tiles
// (16 (tap, c) columns each) and all MT output-channel tiles.
struct WgGeom {
  int LH, LW, OWP, Kpad, nk, src_elems, slack;
};
__host__ __device__ inline WgGeom wg_geom(const ImgWgradArgs& a, int CS) {
  WgGeom g;
  g.LH = (a.OH - 1) * a.stride + a.KH;
  g.LW = (a.OW - 1) * a.stride + a.KW;
  g.OWP = CS <= 4 ? 8 : 4;  // 8 consecutive k (few-channel A fragment) / 4 (tr read) in one row
  while (g.OWP < a.OW) g.OWP <<= 1;
  g.Kpad = ((a.OH * g.OWP + 31) / 32) * 32;
  g.nk = g.Kpad / 32;
  g.src_elems = g.LH * g.LW * CS;
  // dummy pixels (ox in [OW, OWP), rows >= OH) read past the image: zero slack
  const int rows_extra = g.Kpad / g.OWP - a.OH + 1;
  g.slack = ((rows_extra * a.stride + 1) * g.LW + g.OWP * a.stride) * CS;
  g.slack = (g.slack + 7) / 8 * 8;
  return g;
}

// dY image [Kpad][NP] in pixel order k = oy*OWP + ox (dummy pixels and
// channels >= N zero), optionally un-pooled on load from (dy_pooled, dy_argmax).
template <int NP>
__device__ __forceinline__ void stage_dy(bf16* dimg, const ImgWgradArgs& a, const WgGeom& G, long b) {
  const int cpp = NP / 8, total = G.Kpad * cpp;
  const float inv_owp = 1.f / (float)G.OWP;
#pragma unroll 4
  for (int i = threadIdx.x; i < total; i += IC_THREADS) {
    const int ch = (i % cpp) * 8, pix = i / cpp, oy = fdiv(pix, G.OWP, inv_owp), ox = pix - oy * G.OWP;
    u32x4_t v = {0u, 0u, 0u, 0u};
    if (oy < a.OH && ox < a.OW && ch < a.N) {
      if (a.dy) {
        v = *reinterpret_cast<const u32x4_t*>(a.dy + ((b * a.OH + oy) * a.OW + ox) * a.N + ch);
      } else {
        const long po = ((b * (a.OH >> 1) + (oy >> 1)) * (a.OW >> 1) + (ox >> 1)) * a.N + ch;
        const u32x4_t pv = *reinterpret_cast<const u32x4_t*>(a.dy_pooled + po);
        const u32x2_t am = *reinterpret_cast<const u32x2_t*>(a.dy_argmax + po);
        const uint32_t qq = (uint32_t)(((oy & 1) << 1) | (ox & 1));
#pragma unroll
        for (int w = 0; w < 4; ++w) {
          const uint32_t x = (am[w >> 1] ^ (qq * 0x01010101u)) >> (16 * (w & 1));
          const uint32_t lo_ok = (x & 0xffu) == 0u ? 0x0000ffffu : 0u;
          const uint32_t hi_ok = (x & 0xff00u) == 0u ? 0xffff0000u : 0u;
          v[w] = pv[w] & (lo_ok | hi_ok);
        }
      }
    }
    reinterpret_cast<u32x4_t*>(dimg)[i] = v;
  }
}

template <int MT, int CT>
__global__ __launch_bounds__(IC_THREADS) void imgwgrad_kernel(ImgWgradArgs a) {
  extern __shared__ __attribute__((aligned(16))) bf16 smem[];
  const int CS = a.CS;
  const WgGeom G = wg_geom(a, CS);
  constexpr int NP = MT * 16;
  bf16* simg = smem;
  bf16* dimg = smem + G.src_elems + G.slack;  // [Kpad][NP]
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int g = lane >> 4, i16 = lane & 15, q = i16 >> 2, p4 = i16 & 3;
  const int T = a.KH * a.KW, KC = T * CS;
  const int col_tiles = (KC + 15) >> 4;
  const int ct0 = blockIdx.y * 4 * CT + wid * CT;

  // per column tile: this lane's B source offset at k-step 0 for both halves
  int boff[CT][2];
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) {
    const int col = (ct0 + ct) * 16 + 4 * p4;
    int tap = col / CS;
    const int c = col - tap * CS;
    tap = tap < T ? tap : T - 1;  // columns >= KC are discarded at the flush
    const int kh = tap / a.KW, kw = tap - kh * a.KW;
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      const int pixk = 8 * g + 4 * half + q;
      const int oy = pixk / G.OWP, ox = pixk - oy * G.OWP;
      boff[ct][half] = ((oy * a.stride + kh) * G.LW + ox * a.stride + kw) * CS + c;
    }
  }
  const int bstep = (32 / G.OWP) * a.stride * G.LW * CS;  // LDS offset advance per k-step
  int aoff[2];
#pragma unroll
  for (int half = 0; half < 2; ++half) aoff[half] = (8 * g + 4 * half + q) * NP + 4 * p4;

  f32x4_t acc[MT][CT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < CT; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  float dbacc[MT] = {};
  const bool do_db = a.db && blockIdx.y == 0 && wid == 0;

  for (int im = 0; im < a.imgs_per_block; ++im) {
    const long b = (long)blockIdx.x * a.imgs_per_block + im;
    if (b >= a.B) break;
    __syncthreads();  // previous image fully consumed
    stage_image(simg, G.LH, G.LW, a.pad, a.SH, a.SW, CS, a.src, nullptr, nullptr, b, G.slack);
    stage_dy<NP>(dimg, a, G, b);
    __syncthreads();
    for (int s = 0; s < G.nk; ++s) {
      bf16x8_t af[MT];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        // never mask a transposing read per lane: its data was addressed by other lanes
        const s16x4_t h0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            LDS_PTR(s16x4_t, dimg + s * 32 * NP + aoff[0] + mt * 16));
        const s16x4_t h1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            LDS_PTR(s16x4_t, dimg + s * 32 * NP + aoff[1] + mt * 16));
        const s16x8_t v = {h0[0], h0[1], h0[2], h0[3], h1[0], h1[1], h1[2], h1[3]};
        af[mt] = __builtin_bit_cast(bf16x8_t, v);
      }
      if (do_db) {
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
          const s16x8_t v = __builtin_bit_cast(s16x8_t, af[mt]);
          float sum = 0.f;
#pragma unroll
          for (int e = 0; e < 8; ++e) sum += bf2f((bf16)v[e]);
          dbacc[mt] += sum;
        }
      }
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) {
        if (ct0 + ct >= col_tiles) break;  // wave-uniform
        const s16x4_t h0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4_t, simg + boff[ct][0] + s * bstep));
        const s16x4_t h1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4_t, simg + boff[ct][1] + s * bstep));
        const s16x8_t v = {h0[0], h0[1], h0[2], h0[3], h1[0], h1[1], h1[2], h1[3]};
        const bf16x8_t bfr = __builtin_bit_cast(bf16x8_t, v);
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) acc[mt][ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mt], bfr, acc[mt][ct], 0, 0, 0);
      }
    }
  }
  // flush: row = dY channel mt*16 + (lane>>4)*4 + j, col = tap*CS + c = dW column
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
      const int col = (ct0 + ct) * 16 + (lane & 15);
      if (ct0 + ct >= col_tiles || col >= KC) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = mt * 16 + (lane >> 4) * 4 + j;
        if (n < a.N) atomicAdd(a.dw + (long)n * KC + col, acc[mt][ct][j] * a.scale);
      }
    }
  if (do_db) {
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      float v = dbacc[mt];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      const int n = mt * 16 + (lane & 15);
      if (lane < 16 && n < a.N) atomicAdd(a.db + n, v * a.scale);
    }
  }
}

// Few-channel source (CS <= 4, K = T*CS <= 32):
// C[k = (tap, c)][n] = sum_pixel X[pixel + tap][c] * dY[pixel][n].
// A = shifted-image rows (k, 8 consecutive pixels of one output row: 8
// scalar LDS reads at per-lane constant (tap, c) offsets), B = dY image through
// the transposing read.  The 4 waves split the k-steps and reduce through LDS, so
// a workgroup issues one set of N*T global atomics for all its images.
template <int NC>
__global__ __launch_bounds__(IC_THREADS) void imgwgrad1_kernel(ImgWgradArgs a) {
  extern __shared__ __attribute__((aligned(16))) bf16 smem[];
  const int CS = a.CS;
  const WgGeom G = wg_geom(a, CS);
  constexpr int NP = NC * 16;
  bf16* simg = smem;
  const int soff = (G.src_elems + G.slack + 7) / 8 * 8;
  bf16* dimg = smem + soff;                                   // [Kpad][NP]
  float* red = reinterpret_cast<float*>(dimg + G.Kpad * NP);  // [32 taps][NP] + db[NP]
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int g = lane >> 4, i16 = lane & 15, q = i16 >> 2, p4 = i16 & 3;
  const int K = a.KH * a.KW * CS;
  for (int i = threadIdx.x; i < 33 * NP; i += IC_THREADS) red[i] = 0.f;

  int toff[2];
#pragma unroll
  for (int rt = 0; rt < 2; ++rt) {
    const int k = rt * 16 + i16, tap = k / CS, c = k - tap * CS, kh = tap / a.KW;
    toff[rt] = k < K ? (kh * G.LW + (tap - kh * a.KW)) * CS + c : 0;  // rows >= K are dropped at the flush
  }
  // this lane's 8 pixels at k-step s: k = 32s + 8g + j, one output row (OWP >= 8)
  const int k0 = 8 * g, oy0 = k0 / G.OWP, ox0 = k0 - oy0 * G.OWP;
  const int apix0 = oy0 * a.stride * G.LW + ox0 * a.stride;
  const int astep = (32 / G.OWP) * a.stride * G.LW;
  int boff[2];
#pragma unroll
  for (int half = 0; half < 2; ++half) boff[half] = (8 * g + 4 * half + q) * NP + 4 * p4;

  f32x4_t acc[2][NC];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < NC; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  float dbacc[NC] = {};

  for (int im = 0; im < a.imgs_per_block; ++im) {
    const long b = (long)blockIdx.x * a.imgs_per_block + im;
    if (b >= a.B) break;
    __syncthreads();
    stage_image_small(simg, G.LH, G.LW, CS, a.pad, a.SH, a.SW, a.src + b * a.SH * a.SW * CS, G.slack);
    stage_dy<NP>(dimg, a, G, b);
    __syncthreads();
    for (int s = wid; s < G.nk; s += 4) {
      bf16x8_t bfr[NC];
#pragma unroll
      for (int ct = 0; ct < NC; ++ct) {
        const s16x4_t h0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4_t, dimg + s * 32 * NP + boff[0] + ct * 16));
        const s16x4_t h1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4_t, dimg + s * 32 * NP + boff[1] + ct * 16));
        const s16x8_t v = {h0[0], h0[1], h0[2], h0[3], h1[0], h1[1], h1[2], h1[3]};
        bfr[ct] = __builtin_bit_cast(bf16x8_t, v);
        if (a.db) {
          float sum = 0.f;
#pragma unroll
          for (int e = 0; e < 8; ++e) sum += bf2f((bf16)v[e]);
          dbacc[ct] += sum;
        }
      }
      const int apix = apix0 + s * astep;
#pragma unroll
      for (int rt = 0; rt < 2; ++rt) {
        s16x8_t av;
#pragma unroll
        for (int j = 0; j < 8; ++j) av[j] = (short)simg[(apix + j * a.stride) * CS + toff[rt]];
        const bf16x8_t af = __builtin_bit_cast(bf16x8_t, av);
#pragma unroll
        for (int ct = 0; ct < NC; ++ct) acc[rt][ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfr[ct], acc[rt][ct], 0, 0, 0);
      }
    }
  }
  // cross-wave reduction in LDS, then one global atomic per (n, k)
#pragma unroll
  for (int rt = 0; rt < 2; ++rt)
#pragma unroll
    for (int ct = 0; ct < NC; ++ct)
#pragma unroll
      for (int j = 0; j < 4; ++j) atomicAdd(red + (rt * 16 + g * 4 + j) * NP + ct * 16 + i16, acc[rt][ct][j]);
  if (a.db) {
#pragma unroll
    for (int ct = 0; ct < NC; ++ct) {
      float v = dbacc[ct];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      if (lane < 16) atomicAdd(red + 32 * NP + ct * 16 + lane, v);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < K * a.N; i += IC_THREADS) {
    const int n = i / K, k = i - n * K;
    atomicAdd(a.dw + i, red[k * NP + n] * a.scale);
  }
  if (a.db)
    for (int n = threadIdx.x; n < a.N; n += IC_THREADS) atomicAdd(a.db + n, red[32 * NP + n] * a.scale);
}

static int wg_nt(int N) { return N <= 16 ? 1 : (N <= 32 ? 2 : 4); }

static size_t wg_lds(const ImgWgradArgs& a) {
  const int MT = wg_nt(a.N);
  if (a.CS <= 4) {
    const WgGeom G = wg_geom(a, a.CS);
    return ((size_t)(G.src_elems + G.slack + 7) / 8 * 8 + (size_t)G.Kpad * MT * 16) * sizeof(bf16) +
           33 * MT * 16 * sizeof(float);
  }
  const WgGeom G = wg_geom(a, a.CS);
  return ((size_t)G.src_elems + G.slack + (size_t)G.Kpad * MT * 16) * sizeof(bf16);
}

bool imgwgrad_supported(const ImgWgradArgs& a) {
  if (a.N > 64 || a.OW > 32) return false;
  if (a.CS <= 4) {
    if (a.KH * a.KW * a.CS > 32) return false;
  } else if (a.CS % 8) {
    return false;
  }
  return wg_lds(a) <= 150 * 1024;
}

// images per workgroup: enough workgroups to fill the chip, but >= min_ipb
// images each to amortise the flush atomics
static int wg_ipb(int B, int blocks_target, int min_ipb) {
  int ipb = (B + blocks_target - 1) / blocks_target;
  return ipb < min_ipb ? min_ipb : ipb;
}

template <int MT, int CT>
static void launch_wg(const ImgWgradArgs& a0, hipStream_t s) {
  ImgWgradArgs a = a0;
  const size_t lds = wg_lds(a);
  const int KC = a.KH * a.KW * a.CS;
  const int col_tiles = (KC + 15) / 16;
  const int slabs = (col_tiles + 4 * CT - 1) / (4 * CT);
  a.imgs_per_block = wg_ipb(a.B, (1024 + slabs - 1) / slabs, 4);
  const int groups = (a.B + a.imgs_per_block - 1) / a.imgs_per_block;
  auto k = imgwgrad_kernel<MT, CT>;
  if (lds > 64 * 1024) (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(k, dim3(groups, slabs), dim3(IC_THREADS), lds, s, a);
}

template <int NC>
static void launch_wg1(const ImgWgradArgs& a0, hipStream_t s) {
  ImgWgradArgs a = a0;
  const size_t lds = wg_lds(a);
  // one image per workgroup up to 512 images (ResNet-20 stem, B = 256: 16.4 us vs 18.5 at two,
  // 27.0 at four - profiles/r5_resnet20_kernels.txt; DTFE_DIAG iw1=<n> forces n)
  static const int ipb_diag = diag_bits("iw1");
  a.imgs_per_block = ipb_diag > 0 ? ipb_diag : wg_ipb(a.B, 512, 1);
  const int groups = (a.B + a.imgs_per_block - 1) / a.imgs_per_block;
  auto k = imgwgrad1_kernel<NC>;
  if (lds > 64 * 1024) (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(k, dim3(groups), dim3(IC_THREADS), lds, s, a);
}

void launch_imgwgrad(const ImgWgradArgs& a, hipStream_t s) {
  if (!imgwgrad_supported(a)) throw std::runtime_error("imgwgrad: shape not supported");
  if (a.bns.stats && a.CS <= 4) throw std::runtime_error("imgwgrad: BN-on-load needs the persistent kernel");
  if (a.CS <= 4) {
    if (!a.src) throw std::runtime_error("imgwgrad: few-channel path needs src");
    if (launch_conv1_copies_wgrad(a, s)) return;
    switch (wg_nt(a.N)) {
      case 1: launch_wg1<1>(a, s); break;
      case 2: launch_wg1<2>(a, s); break;
      default: launch_wg1<4>(a, s); break;
    }
    return;
  }
  if (launch_imgwgrad_persistent(a, s)) return;
  if (a.bns.stats) throw std::runtime_error("imgwgrad: BN-on-load needs the persistent kernel (B >= 128)");
  if (a.N <= 16) launch_wg<1, 8>(a, s);
  else if (a.N <= 32) launch_wg<2, 6>(a, s);
  else launch_wg<4, 4>(a, s);
}

}  // namespace dtfe
