// Persistent whole-image convolution: weights resident in LDS, images streamed.
//
// The one-image-per-workgroup kernel (imgconv.hip) re-fetched its weight
// fragments from L2 for every image and exposed the L2 latency every k-step
// (rocprof: conv2 fwd at ~15 % MFMA utilisation).  Here one workgroup per CU
// stages the whole weight matrix [N][K] into LDS once (<= ~104 KB for the
// MNIST/CIFAR layers), then loops over its share of the batch:
//
//   write image b (prefetched registers) -> LDS    barrier
//   issue global loads of image b+grid into registers
//   MFMA k-loop over image b from LDS (A: image pixel+tap, B: weights), epilogue
//   barrier
//
// so the next image's HBM latency hides under this image's MFMAs.
//
// Bank conflicts (MI355X_MICROARCH.md §LDS: ds_read_b128 is serviced in the
// lane groups {0-3,12-15,20-27}, {4-11,16-19,28-31}, ... - rows 0-3/12-15 of a
// fragment at one 16-byte chunk, rows 4-11 at the next):
//  * weight rows are KP elements apart with KP*2 = 32 (mod 64) bytes: rows r
//    land on slot 2r (+1 for rows 4-11) - all 16 distinct;
//  * output rows are ordered in 2x2 windows (pool order) with the windows of
//    a 16-row tile permuted (0,2,3,1) over its 4 row quads, and the LDS pixel
//    stride PS / row pitch LWP are chosen on the host by scoring every
//    candidate with that lane-group model (MNIST conv2: 8.6 -> ~1.2 modelled
//    extra cycles per A read).
// Waves form a WM x WN grid: WM over 16-row output tiles, WN over n-tiles (NT
// per wave).  The zero border of the padded image never changes and is written
// once.  With flip_taps (data gradient) the taps are flipped while staging the
// weights, so the inner loop is the same for fwd and dgrad.
#include "imgconv.h"
#include "igemm.h"

#include <algorithm>
#include <cstdlib>
#include <map>
#include <mutex>
#include <stdexcept>
#include <tuple>
#include <type_traits>

namespace dtfe {

namespace {

// compile-time loop: f(std::integral_constant<int, I>{}) for I in [B, E)
template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

struct PGeom {
  int LH, LW;     // LDS image extent (pixels)
  int LWP;        // LDS row pitch (pixels, >= LW)
  int PS;         // LDS pixel stride (elements, >= CS)
  int K, KP;      // reduction length, LDS weight row stride (elements, zero padded past K)
  int NTOT;       // weight rows staged (N rounded up to the wave grid's columns)
  int img_off;    // element offset of the image region
  int slack;      // zero elements after the image (k walk past the last tap when K % 32 != 0)
  int nchunks;    // 16-byte source chunks per image (pooled chunks for a pooled source)
  int npf;        // chunks per thread
  int blocked;    // output rows in 2x2-window order (OH, OW even)
  int stage_out;  // un-pooled output staged in LDS [OH*OW][N] after the image, stored as 16-B rows
  int lg_ow;      // log2(OW) when OW is a power of two (row_pixel by shifts), else -1
};

// row_pixel for OW = 2^lg: shifts and masks instead of two integer divisions by a runtime OW (each
// ~30 VALU; the staged epilogue evaluates it per output value - rocprof: ~70 VALU per MFMA in the
// stage-1 ResNet-20 conv, profiles/r5_resnet20_kernels.txt)
__device__ __forceinline__ bool row_pixel_p2(int m, int OH, int lg, int blocked, int& oy, int& ox) {
  if (blocked) {
    const int t = m >> 4, quad = (m >> 2) & 3, q = m & 3;
    const int w = t * 4 + (quad == 0 ? 0 : quad == 1 ? 2 : quad == 2 ? 3 : 1);
    if (w >= (OH >> 1) << (lg - 1)) return false;
    oy = 2 * (w >> (lg - 1)) + (q >> 1);
    ox = 2 * (w & ((1 << (lg - 1)) - 1)) + (q & 1);
    return true;
  }
  if (m >= OH << lg) return false;
  oy = m >> lg;
  ox = m & ((1 << lg) - 1);
  return true;
}

// output row m of an image -> (oy, ox); false for padding rows of the last tile.
// Blocked order: row quad `quad` of 16-row tile t is window t*4 + {0,2,3,1}[quad].
__host__ __device__ inline bool row_pixel(int m, int OH, int OW, int blocked, int& oy, int& ox) {
  if (blocked) {
    const int t = m >> 4, quad = (m >> 2) & 3, q = m & 3;
    const int w = t * 4 + (quad == 0 ? 0 : quad == 1 ? 2 : quad == 2 ? 3 : 1);
    const int POW = OW >> 1;
    if (w >= (OH >> 1) * POW) return false;
    oy = 2 * (w / POW) + (q >> 1);
    ox = 2 * (w % POW) + (q & 1);
    return true;
  }
  if (m >= OH * OW) return false;
  oy = m / OW;
  ox = m % OW;
  return true;
}

// CSC != 0: a 3x3 conv over CSC source channels (ResNet-20) with the k walk in closed form - step s's
// A offset from k = 32 s + 8 g by divisions by compile-time constants - and the step loop unrolled
// with its fragment reads pinned one step ahead of the MFMAs.  The runtime walk (a per-step while
// loop under exec masking, ~35 instructions and the LDS read latency exposed per 2 MFMAs in the
// stage-1 instance) stays for every other shape.
template <int NT, int RT, int WM, int WN, int NPF, bool POOLED, bool BNX = false, int CSC = 0>
__global__ __launch_bounds__(64 * WM* WN) void imgconv_persist_kernel(ImgConvArgs a, PGeom G) {
  constexpr int THREADS = 64 * WM * WN;
  extern __shared__ __attribute__((aligned(16))) bf16 lds[];
  bf16* wl = lds;
  bf16* img = lds + G.img_off;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid % WM, wn = wid / WM;
  const int T = a.KH * a.KW, CS = a.CS, PS = G.PS, LWP = G.LWP;
  const int CPP = CS / 8;
  auto rp = [&](int m, int blocked, int& oy, int& ox) {
    return G.lg_ow > 0 ? row_pixel_p2(m, a.OH, G.lg_ow, blocked, oy, ox) : row_pixel(m, a.OH, a.OW, blocked, oy, ox);
  };
  // BatchNorm + ReLU of the source on staging (a.bns): this thread's chunks are channels
  // [(tid % CPP) * 8, +8) of every pixel (THREADS % CPP == 0); workgroup 0 saves the statistics
  // (a compile-time instance: the plain kernel keeps its registers and schedule)
  constexpr bool bnx = BNX && !POOLED;
  float bsc[8], bsh[8];
  if constexpr (bnx) {
    bn_src_coeffs(a.bns, a.src, CS, (tid % CPP) * 8, bsc, bsh);
    if (blockIdx.x == 0) bn_src_save(a.bns, a.src, CS, THREADS);
  }
  auto stamp = [&](int k) {  // phase stamps (diagnostics: a.tstamp, bench/resnet20_kernels.py --phases)
    if (a.tstamp && tid == 0) a.tstamp[blockIdx.x * 8 + k] = __builtin_amdgcn_s_memrealtime();
  };
  stamp(0);

  // ---- one-time: zero image region (+ slack), stage (possibly tap-flipped) weights
  for (int i = tid; i < (G.LH * LWP * PS + G.slack) / 8; i += THREADS)
    reinterpret_cast<u32x4_t*>(img)[i] = u32x4_t{0u, 0u, 0u, 0u};
  {
    // 8 loads in flight per thread: the ~100 KB prologue costs a few latencies, not one per chunk
    const int kc_row = G.KP / 8, total = G.NTOT * kc_row;
    // (n, chunk) of i = i0 + u * THREADS stepped incrementally: one runtime division per thread, not
    // one per chunk (~30 VALU each)
    const int dn = THREADS / kc_row, dr = THREADS - dn * kc_row;
    int n_i = tid / kc_row, r_i = tid - n_i * kc_row;
    for (int i0 = tid; i0 < total; i0 += 8 * THREADS) {
      u32x4_t v[8];
      int off[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int i = i0 + u * THREADS;
        const int n = n_i, k = r_i * 8;
        n_i += dn;
        r_i += dr;
        if (r_i >= kc_row) {
          r_i -= kc_row;
          ++n_i;
        }
        off[u] = i < total ? n * G.KP + k : -1;
        v[u] = u32x4_t{0u, 0u, 0u, 0u};
        if (i < total && n < a.N && k < G.K && !(a.diag & 8)) {
          int sk = k;
          if (a.flip_taps) {
            const int tap = k / CS;
            sk = (T - 1 - tap) * CS + (k - tap * CS);
          }
          v[u] = *reinterpret_cast<const u32x4_t*>(a.w + (long)n * G.K + sk);
        }
      }
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (off[u] >= 0) *reinterpret_cast<u32x4_t*>(wl + off[u]) = v[u];
    }
  }

  // ---- per-thread source chunks: LDS destinations are the same for every image
  int dst[NPF];
#pragma unroll
  for (int j = 0; j < NPF; ++j) {
    const int i = tid + j * THREADS;
    dst[j] = -1;
    if (i < G.nchunks) {
      const int pix = i / CPP, cc = i - pix * CPP;
      int sy, sx;
      if (POOLED) {
        const int PW = a.SW >> 1, py = pix / PW, px = pix - py * PW;
        sy = 2 * py;
        sx = 2 * px;
      } else {
        sy = pix / a.SW;
        sx = pix - sy * a.SW;
      }
      const int dil = a.dil > 1 ? a.dil : 1;
      const int ly = sy * dil + a.pad, lx = sx * dil + a.pad;
      // host guarantees pooled windows lie inside the extent; plain pixels outside it are unused
      if (ly < G.LH && lx < G.LW) dst[j] = (ly * LWP + lx) * PS + cc * 8;
    }
  }
  u32x4_t pf[NPF];
  u32x2_t pam[NPF];
  auto load_src = [&](long b) {
#pragma unroll
    for (int j = 0; j < NPF; ++j) {
      const long i = tid + j * THREADS;
      if (i < G.nchunks) {
        const long off = b * G.nchunks * 8 + i * 8;
        if (POOLED) {
          pf[j] = *reinterpret_cast<const u32x4_t*>(a.src_pooled + off);
          pam[j] = *reinterpret_cast<const u32x2_t*>(a.src_argmax + off);
        } else {
          pf[j] = *reinterpret_cast<const u32x4_t*>(a.src + off);
        }
      }
    }
  };
  auto write_src = [&]() {
#pragma unroll
    for (int j = 0; j < NPF; ++j) {
      if (dst[j] < 0) continue;
      if (!POOLED) {
        *reinterpret_cast<u32x4_t*>(img + dst[j]) = bnx ? bn_relu_chunk(pf[j], bsc, bsh) : pf[j];
      } else {
        u32x4_t v[4];
        unpool4(pf[j], pam[j], v);
#pragma unroll
        for (int q = 0; q < 4; ++q)
          *reinterpret_cast<u32x4_t*>(img + dst[j] + ((q >> 1) * LWP + (q & 1)) * PS) = v[q];
      }
    }
  };

  // ---- per-lane constants of the k walk
  const int g = lane >> 4;
  const int M = a.OH * a.OW, tiles = (M + 15) >> 4;
  const int nk = (G.K + 31) >> 5;
  const int tap0 = (8 * g) / CS, cs0 = 8 * g - tap0 * CS;
  const int kh0 = tap0 / a.KW, kw0 = tap0 - kh0 * a.KW;
  const int toff0 = (kh0 * LWP + kw0) * PS + cs0;
  const int wrap_jump = PS - CS, row_jump = (LWP - a.KW) * PS;
  const bf16* wlane = wl + (wn * NT * 16 + (lane & 15)) * G.KP + 8 * g;

  long b = blockIdx.x;
  if (b < a.B && !(a.diag & 2)) load_src(b);
  __syncthreads();  // zero border before the first interior write
  stamp(1);
  for (; b < a.B; b += gridDim.x) {
    if (!(a.diag & 2)) write_src();
    __syncthreads();
    if (b == blockIdx.x) stamp(2);
    if (b + gridDim.x < a.B && !(a.diag & 2)) load_src(b + gridDim.x);
    for (int t0 = wm; t0 < tiles; t0 += WM * RT) {
      int pix[RT];
#pragma unroll
      for (int r = 0; r < RT; ++r) {
        int oy = 0, ox = 0;
        // padding rows read pixel 0 and are dropped by the epilogue
        rp((t0 + WM * r) * 16 + (lane & 15), G.blocked, oy, ox);
        pix[r] = (oy * a.stride * LWP + ox * a.stride) * PS;
      }
      f32x4_t acc[RT][NT];
#pragma unroll
      for (int r = 0; r < RT; ++r)
#pragma unroll
        for (int n = 0; n < NT; ++n) acc[r][n] = f32x4_t{0.f, 0.f, 0.f, 0.f};
      if constexpr (CSC != 0) {
        constexpr int NK = (9 * CSC + 31) / 32, KP = NK * 32 + 16;
        auto toff_of = [&](int st) {
          const int k = 32 * st + 8 * g, tap = k / CSC, kh = tap / 3;
          return (kh * LWP + (tap - 3 * kh)) * PS + (k - tap * CSC);
        };
        u32x4_t fa[2][RT], fb[2][NT];
        {
          const int t = toff_of(0);
#pragma unroll
          for (int n = 0; n < NT; ++n) fb[0][n] = *reinterpret_cast<const u32x4_t*>(wlane + n * 16 * KP);
#pragma unroll
          for (int r = 0; r < RT; ++r) fa[0][r] = *reinterpret_cast<const u32x4_t*>(img + pix[r] + t);
        }
        if (!(a.diag & 4)) static_for<0, NK>([&](auto sc) {
          constexpr int st = decltype(sc)::value, cur = st & 1, nxt = cur ^ 1;
          if constexpr (st + 1 < NK) {
            const int t = toff_of(st + 1);
#pragma unroll
            for (int n = 0; n < NT; ++n)
              fb[nxt][n] = *reinterpret_cast<const u32x4_t*>(wlane + n * 16 * KP + (st + 1) * 32);
#pragma unroll
            for (int r = 0; r < RT; ++r) fa[nxt][r] = *reinterpret_cast<const u32x4_t*>(img + pix[r] + t);
          }
#pragma unroll
          for (int r = 0; r < RT; ++r)
#pragma unroll
            for (int n = 0; n < NT; ++n)
              acc[r][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, fa[cur][r]),
                                                                  __builtin_bit_cast(bf16x8_t, fb[cur][n]), acc[r][n],
                                                                  0, 0, 0);
          // next step's reads ahead of this step's MFMAs (the scheduler would sink them to their use)
          constexpr int nr = st + 1 < NK ? RT + NT : 0;
          if constexpr (nr > 0) __builtin_amdgcn_sched_group_barrier(0x100, nr, 0);
          __builtin_amdgcn_sched_group_barrier(0x8, RT * NT, 0);
        });
      } else {
      // software pipeline: fragments of step s+1 are read while step s's MFMAs run.
      // Past K the weight rows are zero (and the image slack is zero), so no masking.
      int cs = cs0, kw = kw0, toff = toff0;
      u32x4_t af[RT], bfr[NT];
#pragma unroll
      for (int n = 0; n < NT; ++n) bfr[n] = *reinterpret_cast<const u32x4_t*>(wlane + n * 16 * G.KP);
#pragma unroll
      for (int r = 0; r < RT; ++r) af[r] = *reinterpret_cast<const u32x4_t*>(img + pix[r] + toff);
      const int nkk = (a.diag & 4) ? 0 : nk;
      for (int s = 0; s < nkk; ++s) {
        cs += 32;
        toff += 32;
        while (cs >= CS) {
          cs -= CS;
          toff += wrap_jump;
          if (++kw == a.KW) { kw = 0; toff += row_jump; }
        }
        u32x4_t an[RT], bn[NT];
        const int sn = s + 1 < nk ? s + 1 : s;  // last step re-reads (harmless) instead of branching
        const int tn = s + 1 < nk ? toff : toff0;
#pragma unroll
        for (int n = 0; n < NT; ++n) bn[n] = *reinterpret_cast<const u32x4_t*>(wlane + n * 16 * G.KP + sn * 32);
#pragma unroll
        for (int r = 0; r < RT; ++r) an[r] = *reinterpret_cast<const u32x4_t*>(img + pix[r] + tn);
#pragma unroll
        for (int r = 0; r < RT; ++r)
#pragma unroll
          for (int n = 0; n < NT; ++n)
            acc[r][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, af[r]),
                                                                __builtin_bit_cast(bf16x8_t, bfr[n]), acc[r][n], 0, 0, 0);
#pragma unroll
        for (int r = 0; r < RT; ++r) af[r] = an[r];
#pragma unroll
        for (int n = 0; n < NT; ++n) bfr[n] = bn[n];
      }
      }  // (runtime k walk)
      if (b == blockIdx.x && t0 == wm) stamp(3);
      // epilogue: lane holds rows (lane>>4)*4 + j of each tile (one 2x2 window when blocked),
      // column lane&15 of each n-tile
#pragma unroll
      for (int r = 0; r < RT; ++r) {
        const int tile = t0 + WM * r;
        if (tile >= tiles || (a.diag & 1)) break;
        const int m0 = tile * 16 + (lane >> 4) * 4;
#pragma unroll
        for (int n = 0; n < NT; ++n) {
          const int col = (wn * NT + n) * 16 + (lane & 15);
          if (col >= a.N) continue;
          const float bias = a.bias ? a.bias[col] : 0.f;
          const f32x4_t v = acc[r][n];
          if (a.pool) {  // pool implies blocked rows: the quad is one window
            int oy, ox;
            if (!rp(m0, 1, oy, ox)) continue;
            int am = 0;
            float mx = v[0];
#pragma unroll
            for (int j = 1; j < 4; ++j) if (v[j] > mx) { mx = v[j]; am = j; }
            const long o = ((b * (a.OH >> 1) + (oy >> 1)) * (a.OW >> 1) + (ox >> 1)) * a.N + col;
            a.y[o] = f2bf(apply_act(mx + bias, a.act));
            if (a.argmax) a.argmax[o] = (uint8_t)am;
          } else if (G.stage_out) {
            bf16* sy = img + G.LH * LWP * PS + G.slack;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              int oy, ox;
              if (!rp(m0 + j, G.blocked, oy, ox)) continue;
              sy[((oy << G.lg_ow) + ox) * a.N + col] = f2bf(apply_act(v[j] + bias, a.act));
            }
          } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              int oy, ox;
              if (!rp(m0 + j, G.blocked, oy, ox)) continue;
              const long o = ((b * a.OH + oy) * a.OW + ox) * a.N + col;
              float x = apply_act(v[j] + bias, a.act);
              if (a.relu_mask && !(bf2f(a.relu_mask[o]) > 0.f)) x = 0.f;
              a.y[o] = f2bf(x);
            }
          }
        }
      }
    }
    if (b == blockIdx.x) stamp(4);
    if (G.stage_out && !(a.diag & 1)) {
      // the image's [OH*OW][N] output leaves as contiguous 16-B chunks (ReLU'-mask of the data
      // gradient applied here from 16-B mask loads): the per-lane 2-byte scatter cost ~8 of the
      // 19 us of ResNet-20's stage-1 conv (DTFE_DIAG icr=1 ablation, profiles/r5_resnet20_kernels.txt)
      __syncthreads();
      const bf16* sy = img + G.LH * LWP * PS + G.slack;
      const int nch = M * a.N / 8;
      const long ob = b * (long)M * a.N;
      for (int i = tid; i < nch; i += THREADS) {
        u32x4_t v = *reinterpret_cast<const u32x4_t*>(sy + i * 8);
        if (a.relu_mask) {
          const u32x4_t m = *reinterpret_cast<const u32x4_t*>(a.relu_mask + ob + i * 8);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            // keep element where mask > 0 (bf16 bits: positive, non-zero, not NaN)
            const uint32_t ml = m[e] & 0xffffu, mh = m[e] >> 16;
            v[e] = (((ml - 1u) < 0x7f80u) ? (v[e] & 0xffffu) : 0u) | (((mh - 1u) < 0x7f80u) ? (v[e] & 0xffff0000u) : 0u);
          }
        }
        if (a.sc_src) {  // + the shortcut's gradient at its (strided) pixels, in fp32 then one rounding
          const int CPN = a.N >> 3, p = i / CPN, cc = i - p * CPN, oy = p / a.OW, ox = p - oy * a.OW;
          const int st = a.sc_stride;
          if ((oy % st) == 0 && (ox % st) == 0) {
            const long gi = ((b * (a.OH / st) + oy / st) * (long)(a.OW / st) + ox / st) * a.sc_C + cc * 8;
            const u32x4_t gv = *reinterpret_cast<const u32x4_t*>(a.sc_src + gi);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float lo = __uint_as_float(v[e] << 16) + __uint_as_float(gv[e] << 16);
              const float hi = __uint_as_float(v[e] & 0xffff0000u) + __uint_as_float(gv[e] & 0xffff0000u);
              v[e] = pack_bf16x2(lo, hi);
            }
          }
        }
        *reinterpret_cast<u32x4_t*>(a.y + ob + i * 8) = v;
      }
    }
    if (b == blockIdx.x) stamp(5);
    __syncthreads();  // image b fully consumed before the next write
  }
  stamp(6);
}

// ----------------------------------------------------- compile-time geometry
// The same persistent structure with the whole layer geometry as template constants (MNIST
// conv2 forward and data gradient).  rocprof PMC of the runtime-geometry kernel above: 9-14
// VALU instructions per MFMA (the per-step k walk, address adds and fragment register
// copies of a 2-4 MFMA step) - the kernel was VALU-issue bound.  Here the k loop is fully
// unrolled: every fragment read is `ds_read_b128 base + immediate` (tap offsets and weight
// offsets are constants), the double-buffered fragment registers alternate by step parity
// at compile time, and a step costs RT + NT reads, RT x NT MFMAs and no VALU.
// One wave per RT 16-row tiles x all N columns (NT = N/16), WM waves cover the image.
template <int CS, int KH, int KW, int LWP, int PS, int KP, int NT, int RT, int WM, int NPF, bool POOLED, int ACT>
__global__ __launch_bounds__(64 * WM) void imgconv_fixed_kernel(ImgConvArgs a, PGeom G) {
  constexpr int THREADS = 64 * WM;
  constexpr int T = KH * KW, K = T * CS, NK = K / 32, CPP = CS / 8;
  static_assert(K % 32 == 0 && CS % 32 == 0, "whole 32-deep steps within one tap");
  extern __shared__ __attribute__((aligned(16))) bf16 lds[];
  bf16* wl = lds;
  bf16* img = lds + G.img_off;
  const int tid = threadIdx.x, lane = tid & 63, wm = __builtin_amdgcn_readfirstlane(tid >> 6);

  for (int i = tid; i < (G.LH * LWP * PS) / 8; i += THREADS)
    reinterpret_cast<u32x4_t*>(img)[i] = u32x4_t{0u, 0u, 0u, 0u};
  {
    constexpr int kc_row = KP / 8;
    const int total = G.NTOT * kc_row;
    for (int i0 = tid; i0 < total; i0 += 8 * THREADS) {
      u32x4_t v[8];
      int off[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int i = i0 + u * THREADS;
        const int n = i / kc_row, k = (i - n * kc_row) * 8;
        off[u] = i < total ? n * KP + k : -1;
        v[u] = u32x4_t{0u, 0u, 0u, 0u};
        if (i < total && n < a.N && k < K) {
          int sk = k;
          if (a.flip_taps) {
            const int tap = k / CS;
            sk = (T - 1 - tap) * CS + (k - tap * CS);
          }
          v[u] = *reinterpret_cast<const u32x4_t*>(a.w + (long)n * K + sk);
        }
      }
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (off[u] >= 0) *reinterpret_cast<u32x4_t*>(wl + off[u]) = v[u];
    }
  }

  int dst[NPF];
#pragma unroll
  for (int j = 0; j < NPF; ++j) {
    const int i = tid + j * THREADS;
    dst[j] = -1;
    if (i < G.nchunks) {
      const int pix = i / CPP, cc = i - pix * CPP;
      int sy, sx;
      if (POOLED) {
        const int PW = a.SW >> 1, py = pix / PW, px = pix - py * PW;
        sy = 2 * py;
        sx = 2 * px;
      } else {
        sy = pix / a.SW;
        sx = pix - sy * a.SW;
      }
      const int ly = sy + a.pad, lx = sx + a.pad;
      if (ly < G.LH && lx < G.LW) dst[j] = (ly * LWP + lx) * PS + cc * 8;
    }
  }
  u32x4_t pf[NPF];
  u32x2_t pam[NPF];
  auto load_src = [&](long b) {
#pragma unroll
    for (int j = 0; j < NPF; ++j) {
      const long i = tid + j * THREADS;
      if (i < G.nchunks) {
        const long off = b * G.nchunks * 8 + i * 8;
        if (POOLED) {
          pf[j] = *reinterpret_cast<const u32x4_t*>(a.src_pooled + off);
          pam[j] = *reinterpret_cast<const u32x2_t*>(a.src_argmax + off);
        } else {
          pf[j] = *reinterpret_cast<const u32x4_t*>(a.src + off);
        }
      }
    }
  };
  auto write_src = [&]() {
#pragma unroll
    for (int j = 0; j < NPF; ++j) {
      if (dst[j] < 0) continue;
      if (!POOLED) {
        *reinterpret_cast<u32x4_t*>(img + dst[j]) = pf[j];
      } else {
        u32x4_t v[4];
        unpool4(pf[j], pam[j], v);
#pragma unroll
        for (int q = 0; q < 4; ++q)
          *reinterpret_cast<u32x4_t*>(img + dst[j] + ((q >> 1) * LWP + (q & 1)) * PS) = v[q];
      }
    }
  };

  const int g = lane >> 4;
  const int M = a.OH * a.OW, tiles = (M + 15) >> 4;
  const int nout = (POOLED ? M : (M >> 2)) * a.N / 8;  // 16-B chunks of one image's output
  const bf16* wlane = wl + (lane & 15) * KP + 8 * g;
  float biasv[NT];  // loaded once, not once per image in the epilogue
#pragma unroll
  for (int n = 0; n < NT; ++n) biasv[n] = a.bias ? a.bias[n * 16 + (lane & 15)] : 0.f;

  // per-lane geometry is the same for every image: the row -> pixel decode (integer divisions by
  // the runtime OW), the A-fragment bases, the data gradient's output pixels and the forward's
  // pooled staging slots are computed once, not once per image
  const bf16* abase[RT];
  int opix[RT];   // data gradient: output pixel of this lane's column (-1: padding row)
  int ppix[RT];   // forward: pooled pixel of this lane's 2x2 window (-1: padding / past the image)
#pragma unroll
  for (int r = 0; r < RT; ++r) {
    int oy = 0, ox = 0;
    // tiles past the image (a wave's last r) multiply pixel 0 and are dropped by the epilogue:
    // no lane-divergent guards inside the k loop
    const bool ok = row_pixel((wm + WM * r) * 16 + (lane & 15), a.OH, a.OW, G.blocked, oy, ox);
    abase[r] = img + (ok ? (oy * LWP + ox) * PS : 0) + 8 * g;
    opix[r] = ok ? oy * a.OW + ox : -1;
    const int tile = wm + WM * r;
    int py = 0, px = 0;
    const bool pok = tile < tiles && row_pixel(tile * 16 + (lane >> 4) * 4, a.OH, a.OW, 1, py, px);
    ppix[r] = pok ? (py >> 1) * (a.OW >> 1) + (px >> 1) : -1;
  }

  long b = blockIdx.x;
  if (b < a.B) load_src(b);
  __syncthreads();
  for (; b < a.B; b += gridDim.x) {
    if (!(a.diag & 2) || b == blockIdx.x) write_src();
    __syncthreads();
    if (b + gridDim.x < a.B && !(a.diag & 2)) load_src(b + gridDim.x);
    // Data gradient (POOLED source): the MFMA operands are swapped, D = W . patch^T, so a lane's
    // accumulator holds 4 consecutive channels (4g..4g+3 of each n-tile) of ONE output pixel
    // (column lane & 15): the epilogue is one 8-B masked store per n-tile straight to HBM - no
    // LDS staging, no scattered 2-byte writes, no extra barriers (rocprof ablation of the staged
    // version: ~14 us of the 47 us B=1024 launch).  The lane's ReLU-mask words are in flight
    // during the k loop.
    u32x2_t mk[RT][NT];
    if constexpr (POOLED) {
#pragma unroll
      for (int r = 0; r < RT; ++r) {
#pragma unroll
        for (int n = 0; n < NT; ++n) {
          mk[r][n] = u32x2_t{0x3f803f80u, 0x3f803f80u};  // bf16 1.0: no mask
          if (opix[r] >= 0 && a.relu_mask)
            mk[r][n] = *reinterpret_cast<const u32x2_t*>(a.relu_mask + (b * M + opix[r]) * (long)a.N + n * 16 + 4 * g);
        }
      }
    }
    f32x4_t acc[RT][NT];
#pragma unroll
    for (int r = 0; r < RT; ++r)
#pragma unroll
      for (int n = 0; n < NT; ++n) acc[r][n] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    // fragments are fetched PF steps ahead (ring of PF + 1 register sets): LDS read latency,
    // not bandwidth, bounds this loop
    constexpr int PF = 2;
    u32x4_t fa[PF + 1][RT], fb[PF + 1][NT];
    auto fetch = [&](auto sc) {
      constexpr int st = decltype(sc)::value;
      constexpr int k0 = 32 * st, tap = k0 / CS, cs = k0 - tap * CS;
      constexpr int toff = ((tap / KW) * LWP + (tap % KW)) * PS + cs;
      constexpr int buf = st % (PF + 1);
#pragma unroll
      for (int r = 0; r < RT; ++r) fa[buf][r] = *reinterpret_cast<const u32x4_t*>(abase[r] + toff);
#pragma unroll
      for (int n = 0; n < NT; ++n) fb[buf][n] = *reinterpret_cast<const u32x4_t*>(wlane + n * 16 * KP + k0);
    };
    static_for<0, PF>([&](auto sc) {
      if constexpr (decltype(sc)::value < NK) fetch(sc);
    });
    if (!(a.diag & 4)) static_for<0, NK>([&](auto sc) {
      constexpr int st = decltype(sc)::value;
      if constexpr (st + PF < NK) fetch(std::integral_constant<int, st + PF>{});
      constexpr int buf = st % (PF + 1);
#pragma unroll
      for (int r = 0; r < RT; ++r) {
#pragma unroll
        for (int n = 0; n < NT; ++n) {
          if constexpr (POOLED)  // D[channel][pixel]
            acc[r][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, fb[buf][n]),
                                                                __builtin_bit_cast(bf16x8_t, fa[buf][r]), acc[r][n],
                                                                0, 0, 0);
          else  // D[pixel][channel]
            acc[r][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, fa[buf][r]),
                                                                __builtin_bit_cast(bf16x8_t, fb[buf][n]), acc[r][n],
                                                                0, 0, 0);
        }
      }
      // Pin the interleave: the RT + NT reads of step st + PF spread between step st's MFMAs.
      // Without it the scheduler sinks every read to just before its consumer (one lgkmcnt wait
      // per MFMA pair), leaving the MFMA pipe ~38 % busy (rocprof SQ_VALU_MFMA_BUSY_CYCLES).
      constexpr int nm = RT * NT, nr = (st + PF < NK) ? RT + NT : 0;
      static_for<0, nm>([&](auto ic) {
        constexpr int i = decltype(ic)::value, r0 = i * nr / nm, r1 = (i + 1) * nr / nm;
        if constexpr (r1 > r0) __builtin_amdgcn_sched_group_barrier(0x100, r1 - r0, 0);
        __builtin_amdgcn_sched_group_barrier(0x8, 1, 0);
      });
    });
    // Epilogue through LDS: the per-lane results are scattered 2-byte (and 1-byte argmax) values,
    // so they are staged in LDS in the output's own layout and leave as 16-B row-contiguous
    // stores (each image's output is one contiguous block).  rocprof ablation of the direct
    // scattered stores: ~2 us per image per CU, a quarter of the forward kernel.
    if constexpr (!POOLED) {
      // forward (+bias, act, 2x2 max-pool, argmax): stage [M/4][N] values + [M/4][N] argmax bytes
      // in the dedicated region after the image; the next image's staging is two barriers away
      bf16* sy = img + G.LH * LWP * PS;
      uint8_t* sa = reinterpret_cast<uint8_t*>(sy + (M >> 2) * a.N);
#pragma unroll
      for (int r = 0; r < RT; ++r) {
        if (ppix[r] < 0 || (a.diag & 1)) continue;
        const int pp = ppix[r];
#pragma unroll
        for (int n = 0; n < NT; ++n) {
          const int col = n * 16 + (lane & 15);
          const f32x4_t v = acc[r][n];
          int am = 0;
          float mx = v[0];
#pragma unroll
          for (int j = 1; j < 4; ++j) if (v[j] > mx) { mx = v[j]; am = j; }
          sy[pp * a.N + col] = f2bf(apply_act(mx + biasv[n], ACT));
          sa[pp * a.N + col] = (uint8_t)am;
        }
      }
      __syncthreads();
      const int ny = nout, na = nout / 2;  // 16-B chunks of values / argmax bytes
      const long pb = b * (M >> 2) * a.N;
      for (int i = tid; i < ny + na; i += THREADS) {
        if (i < ny) {
          *reinterpret_cast<u32x4_t*>(a.y + pb + i * 8) = *reinterpret_cast<const u32x4_t*>(sy + i * 8);
        } else if (a.argmax) {
          const int k = i - ny;
          *reinterpret_cast<u32x4_t*>(a.argmax + pb + k * 16) = *reinterpret_cast<const u32x4_t*>(sa + k * 16);
        }
      }
    } else {
      // data gradient (ReLU'-masked, no pool): lane = one pixel, 4 consecutive channels per n-tile
#pragma unroll
      for (int r = 0; r < RT; ++r) {
        if (opix[r] < 0 || (a.diag & 1)) continue;
        bf16* yp = a.y + (b * M + opix[r]) * (long)a.N + 4 * g;
#pragma unroll
        for (int n = 0; n < NT; ++n) {
          uint32_t w2[2];
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const uint32_t lo = f2bf(apply_act(acc[r][n][2 * h] + biasv[n], ACT));
            const uint32_t hi = f2bf(apply_act(acc[r][n][2 * h + 1] + biasv[n], ACT));
            // keep element e where mask e > 0 (bf16 bits: positive, non-zero, not NaN)
            const uint32_t m = mk[r][n][h], ml = m & 0xffffu, mh = m >> 16;
            w2[h] = (((ml - 1u) < 0x7f80u) ? lo : 0u) | (((mh - 1u) < 0x7f80u) ? (hi << 16) : 0u);
          }
          *reinterpret_cast<u32x2_t*>(yp + n * 16) = u32x2_t{w2[0], w2[1]};
        }
      }
      __syncthreads();  // every wave is done reading the image before the next one is written
    }
  }
}

// ---------------------------------------------------------------- host side
// Extra LDS cycles per A-fragment ds_read_b128 (averaged over the image's tiles)
// for pixel stride PSs (16 B slots) and row pitch LWP, from the lane-group model.
double a_read_conflicts(int PSs, int LWP, int OH, int OW, int stride, int blocked) {
  static const int groups[4][16] = {
      {0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27},
      {4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31},
      {32, 33, 34, 35, 44, 45, 46, 47, 52, 53, 54, 55, 56, 57, 58, 59},
      {36, 37, 38, 39, 40, 41, 42, 43, 48, 49, 50, 51, 60, 61, 62, 63}};
  const int M = OH * OW, tiles = (M + 15) / 16;
  double total = 0;
  for (int t = 0; t < tiles; ++t) {
    int slot[64];
    for (int l = 0; l < 64; ++l) {
      int oy = 0, ox = 0;
      row_pixel(t * 16 + (l & 15), OH, OW, blocked, oy, ox);
      slot[l] = ((oy * stride * LWP + ox * stride) * PSs + (l >> 4)) % 16;
    }
    for (const auto& gr : groups) {
      int cnt[16] = {0}, mx = 0;
      for (int l : gr) mx = std::max(mx, ++cnt[slot[l]]);
      total += mx - 1;
    }
  }
  return total / tiles;
}

PGeom persist_geom(const ImgConvArgs& a, int WN, int NT, int threads) {
  PGeom G;
  G.stage_out = 0;
  G.lg_ow = -1;
  for (int l = 1; l <= 10; ++l)
    if (a.OW == (1 << l)) G.lg_ow = l;
  G.LH = (a.OH - 1) * a.stride + a.KH;
  G.LW = (a.OW - 1) * a.stride + a.KW;
  G.K = a.KH * a.KW * a.CS;
  G.KP = (G.K + 31) / 32 * 32 + 16;  // KP*2 bytes = 32 (mod 64): conflict-free weight fragments
  G.NTOT = WN * NT * 16;
  G.img_off = G.NTOT * G.KP;
  G.blocked = ((a.OH | a.OW) & 1) == 0;
  const bool pooled = a.src == nullptr;
  G.nchunks = (pooled ? (a.SH / 2) * (a.SW / 2) : a.SH * a.SW) * (a.CS / 8);
  G.npf = (G.nchunks + threads - 1) / threads;
  // image layout search (cached per geometry): fewest modelled conflicts within the LDS budget
  static std::mutex mu;
  static std::map<std::tuple<int, int, int, int, int, int, int, int>, std::pair<int, int>> cache;
  const auto key = std::make_tuple(a.OH, a.OW, a.CS, a.stride, G.LH, G.LW, G.img_off, (int)(G.K % 32 != 0));
  std::lock_guard<std::mutex> lk(mu);
  auto it = cache.find(key);
  if (it == cache.end()) {
    double best = 1e30;
    std::pair<int, int> pick(a.CS, G.LW);
    for (int PSs = a.CS / 8; PSs < a.CS / 8 + 8; ++PSs)
      for (int LWP = G.LW; LWP < G.LW + 12; ++LWP) {
        const long slack = (G.K % 32) ? (long)(LWP + 4) * PSs * 8 : 0;
        const long bytes = ((long)G.img_off + (long)G.LH * LWP * PSs * 8 + slack) * 2;
        if (bytes > 160 * 1024) continue;
        const double c = a_read_conflicts(PSs, LWP, a.OH, a.OW, a.stride, G.blocked) + 1e-7 * bytes;
        if (c < best) { best = c; pick = {PSs * 8, LWP}; }
      }
    it = cache.emplace(key, pick).first;
  }
  G.PS = it->second.first;
  G.LWP = it->second.second;
  G.slack = (G.K % 32) ? (G.LWP + 4) * G.PS : 0;
  return G;
}

size_t persist_lds(const PGeom& G) {
  return ((size_t)G.img_off + (size_t)G.LH * G.LWP * G.PS + G.slack) * sizeof(bf16);
}

template <int NT, int RT, int WM, int WN, bool POOLED>
bool launch_cfg(const ImgConvArgs& a, hipStream_t s, bool* sc_done) {
  constexpr int THREADS = 64 * WM * WN;
  PGeom G = persist_geom(a, WN, NT, THREADS);
  size_t lds = persist_lds(G);
  if (lds > 160 * 1024) return false;
  const size_t stage = (size_t)a.OH * a.OW * a.N * sizeof(bf16);
  G.stage_out = !a.pool && a.N % 8 == 0 && lds + stage <= 160 * 1024 && !(diag_bits("icr") & 16) && G.lg_ow > 0;
  if (G.stage_out) lds += stage;
  const bool sc = a.sc_src && G.stage_out && a.sc_stride >= 1 && a.OH % a.sc_stride == 0 &&
                  a.OW % a.sc_stride == 0 && a.sc_C % 8 == 0 && a.N <= a.sc_C;
  if (a.pool && !G.blocked) return false;
  const int grid = a.B < 256 ? a.B : 256;  // one workgroup per CU, persistent over the batch
  static const int diag = diag_bits("icr");
  ImgConvArgs ad = a;
  ad.diag = diag;
  if (!sc) ad.sc_src = nullptr;
  auto go = [&](auto kern) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(THREADS), lds, s, ad, G);
  };
  if (G.npf < 1 || G.npf > 4) return false;
  if constexpr (!POOLED) {
    // ResNet-20's 3x3 convs: the closed-form k walk (CSC instances; DTFE_DIAG icr=64 -> runtime walk)
    const int csc = a.KH == 3 && a.KW == 3 && G.npf <= 2 && !(diag & 64) &&
                            (a.CS == 16 || a.CS == 32 || a.CS == 64) && G.K == 9 * a.CS &&
                            G.KP == (9 * a.CS + 31) / 32 * 32 + 16
                        ? a.CS : 0;
    if (csc) {
      auto pick = [&](auto cst) {
        constexpr int C = decltype(cst)::value;
        if (a.bns.stats) {
          if (G.npf == 1) go(imgconv_persist_kernel<NT, RT, WM, WN, 1, false, true, C>);
          else go(imgconv_persist_kernel<NT, RT, WM, WN, 2, false, true, C>);
        } else {
          if (G.npf == 1) go(imgconv_persist_kernel<NT, RT, WM, WN, 1, false, false, C>);
          else go(imgconv_persist_kernel<NT, RT, WM, WN, 2, false, false, C>);
        }
      };
      if (csc == 16) pick(std::integral_constant<int, 16>{});
      else if (csc == 32) pick(std::integral_constant<int, 32>{});
      else pick(std::integral_constant<int, 64>{});
      if (sc_done) *sc_done = sc;
      return true;
    }
    if (a.bns.stats) {
      switch (G.npf) {
        case 1: go(imgconv_persist_kernel<NT, RT, WM, WN, 1, false, true>); break;
        case 2: go(imgconv_persist_kernel<NT, RT, WM, WN, 2, false, true>); break;
        case 3: go(imgconv_persist_kernel<NT, RT, WM, WN, 3, false, true>); break;
        default: go(imgconv_persist_kernel<NT, RT, WM, WN, 4, false, true>); break;
      }
      if (sc_done) *sc_done = sc;
      return true;
    }
  } else {
    if (a.bns.stats) return false;
  }
  switch (G.npf) {
    case 1: go(imgconv_persist_kernel<NT, RT, WM, WN, 1, POOLED>); break;
    case 2: go(imgconv_persist_kernel<NT, RT, WM, WN, 2, POOLED>); break;
    case 3: go(imgconv_persist_kernel<NT, RT, WM, WN, 3, POOLED>); break;
    default: go(imgconv_persist_kernel<NT, RT, WM, WN, 4, POOLED>); break;
  }
  if (sc_done) *sc_done = sc;
  return true;
}

}  // namespace

// compile-time-geometry instances (MNIST conv2 forward / data gradient); false if `a` is not one
template <int CS, int KH, int KW, int LWP, int PS, int NT, int RT, int WM, bool POOLED, int ACT>
bool launch_fixed(const ImgConvArgs& a, hipStream_t s) {
  constexpr int K = KH * KW * CS, KP = (K + 31) / 32 * 32 + 16;
  if (a.CS != CS || a.KH != KH || a.KW != KW || a.N != NT * 16 || a.stride != 1 || a.dil > 1) return false;
  if (a.act != ACT) return false;  // the activation is a compile-time constant of the epilogue
  if ((a.src == nullptr) != POOLED) return false;
  // the LDS-staged epilogues: forward = pooled (+ argmax), data gradient = un-pooled
  if (POOLED ? a.pool != 0 : a.pool == 0) return false;
  PGeom G = persist_geom(a, 1, NT, 64 * WM);
  if (G.LWP != LWP || G.PS != PS || G.KP != KP || G.slack != 0) return false;
  const int tiles = (a.OH * a.OW + 15) / 16;
  if (tiles > WM * RT) return false;
  // forward staging region after the image: [M/4][N] bf16 values + [M/4][N] argmax bytes
  const size_t lds = persist_lds(G) + (POOLED ? 0 : (size_t)(a.OH * a.OW / 4) * a.N * 3);
  if (lds > 160 * 1024 || (a.pool && !G.blocked)) return false;
  const int grid = a.B < 256 ? a.B : 256;
  static const int diag = diag_bits("ic");
  ImgConvArgs ad = a;
  ad.diag = diag;
  auto go = [&](auto kern) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * WM), lds, s, ad, G);
  };
  switch (G.npf) {
    case 1: go(imgconv_fixed_kernel<CS, KH, KW, LWP, PS, KP, NT, RT, WM, 1, POOLED, ACT>); return true;
    case 2: go(imgconv_fixed_kernel<CS, KH, KW, LWP, PS, KP, NT, RT, WM, 2, POOLED, ACT>); return true;
    default: return false;
  }
}

bool launch_imgconv_persistent(const ImgConvArgs& a, hipStream_t s, bool* sc_done) {
  if (sc_done) *sc_done = false;
  if (a.CS % 8 || a.N > 64 || a.B < 64) return false;
  if (a.OH == 14 && a.OW == 14 && a.B >= 256 && !a.bns.stats) {
    // compile-time geometry, one 16-row tile per wave (13 waves); 2 / 4 tiles per wave (7 / 4
    // waves) measured slower and were removed in round 3
    if (launch_fixed<32, 5, 5, 20, 48, 4, 1, 13, false, ACT_RELU>(a, s)) return true;  // conv2 forward
    if (launch_fixed<64, 5, 5, 20, 80, 2, 1, 13, true, ACT_NONE>(a, s)) return true;   // conv2 data gradient
  }
  const bool pooled = a.src == nullptr;
  if (pooled && ((a.SH | a.SW) & 1)) return false;
  if (pooled && a.dil > 1) return false;
  {  // pooled windows must lie inside the LDS extent (plain pixels outside it are unused)
    const int LH = (a.OH - 1) * a.stride + a.KH, LW = (a.OW - 1) * a.stride + a.KW;
    if (pooled && (a.SH + a.pad > LH || a.SW + a.pad > LW)) return false;
  }
  // wave grid (measured on MNIST conv2, B=1024): 8 x 2 waves, 4 per SIMD (fwd 48 us, dgrad 68) beat
  // 4 x 2 (48 / 74) and 4 x 1 waves holding every n-tile (fewer LDS reads, but one wave per SIMD
  // exposes the read latency: fwd 48 vs 63 us); the alternatives were removed in round 3
  if (a.N <= 16 && !(diag_bits("icr") & 32))  // one n-tile: a second wave column would only compute padding
    return pooled ? launch_cfg<1, 2, 16, 1, true>(a, s, sc_done) : launch_cfg<1, 2, 16, 1, false>(a, s, sc_done);
  if (a.N <= 32) return pooled ? launch_cfg<1, 2, 8, 2, true>(a, s, sc_done) : launch_cfg<1, 2, 8, 2, false>(a, s, sc_done);
  // small maps (<= 4 row tiles: ResNet-20 stage 3, 8x8): 4 x 2 waves of one tile x 2 n-tiles each -
  // the 8 x 2 grid left half its waves idle and computed a padding tile in the rest (s3 conv 8.98 ->
  // 8.27 us, step -6 us; DTFE_DIAG icr=128 -> the 8 x 2 grid, profiles/r5_resnet20_kernels.txt)
  if (a.OH * a.OW <= 64 && !pooled && a.N <= 64 && !(diag_bits("icr") & 128))
    return launch_cfg<2, 1, 4, 2, false>(a, s, sc_done);
  return pooled ? launch_cfg<2, 2, 8, 2, true>(a, s, sc_done) : launch_cfg<2, 2, 8, 2, false>(a, s, sc_done);
}

}  // namespace dtfe
