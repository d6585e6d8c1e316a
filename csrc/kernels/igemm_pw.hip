// Implicit-GEMM convolutions as persistent, pipelined GEMMs on gfx950 (every one-phase launch of
// igemm.hip: 1x1 and 3x3 forward at any stride, stride-1 data gradients, the strided 1x1 data
// gradient that accumulates onto the shortcut's share).  The 1x1 convs alone are two thirds of
// ResNet-50's conv time (profiles/r3_resnet50_convs_b256.txt: 8.3 of 12.9 ms).
//
//   rows = pixels (b, i, j) of the output grid, k = (tap, channel) over the source; tap t reads
//   source pixel (i*istr + dy[t], j*istr + dx[t]) - a zero page outside the image - and weight
//   tap kt[t]; + BatchNorm statistics of the stored bf16 output per tile (forward)
//
// Against the per-tile implicit-GEMM kernel (igemm.hip) this launch
//   * is persistent: one (or two) workgroups per CU walk a contiguous run of output tiles, and the
//     k-tile stream runs ACROSS tile boundaries - the next tile's first k-tiles are in flight while
//     the current tile's epilogue runs (the 1x1 layers have 1-16 k-tiles per tile, so the per-tile
//     load latency and epilogue were most of their time);
//   * keeps NS-1 k-tiles in flight: an NS-stage LDS ring filled by global_load_lds_dwordx4, counted
//     `s_waitcnt vmcnt(N)` and raw s_barrier (no vmcnt(0) drain per k-tile);
//   * has no per-k-tile im2col math: each row's pixel base pointer and 9-bit tap-validity mask
//     are computed once per tile; a k-tile adds the (wave-uniform, scalar) tap offset and selects
//     the zero page by one mask bit;
//   * runs the MFMAs with the operands swapped (D = W . X^T), so a lane's accumulator holds four
//     consecutive CHANNELS of one pixel: the epilogue stores 8-B bf16 quads straight from
//     registers and the BatchNorm partial sums reduce across 16 lanes by shuffles - no C tile in
//     LDS, no LDS round trip, no barrier but one for the two wave rows' statistics.
//
// LDS images are the igemm.hip ones: [rows][64 k] with 128-B rows, logical 16-B chunk c of row r
// in slot c ^ (r & 7) (the swizzle rides on the DMA's per-lane SOURCE address; the fragment read
// undoes it), so the 16 lanes of a ds_read_b128 quarter hit 16 distinct bank slots.
//
// Replaces Conv2D / Conv2DBackpropInput of the 1x1 ResNet-50 layers (BASELINE.json config 5,
// SURVEY.md K16) and the forward BatchNorm statistics pass (K17).
#include "igemm.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>

namespace dtfe {

namespace {

constexpr int PW_THREADS = 256;
// which one-phase launches take the persistent kernel by default (DTFE_PW overrides):
// 0 none, 1 the data gradients that fold BatchNorm-backward statistics in, 2 all
constexpr int PW_DEFAULT_MODE = 0;
constexpr int PW_BK = 64;

typedef __attribute__((address_space(3))) void lds_void_t;

__device__ __forceinline__ void glds16(const void* g, bf16* lds_piece) {
  __builtin_amdgcn_global_load_lds(g, (lds_void_t*)lds_piece, 16, 0, 0);
}

// The same DMA issued from inline asm (M0 = the wave-uniform LDS destination): invisible to the
// compiler's LDS-DMA alias tracking, which otherwise puts an `s_waitcnt vmcnt(0)` in front of the
// first fragment read of every k-tile of a multi-stage ring (it cannot tell the stage being filled
// from the one being read) and so drains the prefetch.  The caller orders every DMA'd tile with
// its own counted vmcnt wait + barrier; the compiler's own waits stay conservative (these DMAs
// are always older than the loads it counts).
__device__ __forceinline__ void glds16_async(const void* g, bf16* lds_piece) {
  const uint32_t l = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)lds_piece);
  asm volatile("global_load_lds_dwordx4 %0, off" ::"v"(g), "{m0}"(l) : "memory");
}

// exact m / d for 0 <= m < 2^24 through a float reciprocal
__device__ __forceinline__ int pdiv(int m, int d, float inv_d) {
  int q = (int)((float)m * inv_d);
  const int r = m - q * d;
  q += (r >= d) - (r < 0);
  return q;
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

template <int BM, int BN, int NS>
constexpr int pw_smem_el() {
  return NS * (BM + BN) * PW_BK + 2 * 4 * BN * 2;  // ring + per-wave-row statistics (4 floats / channel)
}

// row m of the RH x RW grid -> (b, i, j)
__device__ __forceinline__ void pw_rc(int m, int RH, int RW, float inv_rw, float inv_rh, int& b, int& i, int& j) {
  const int t = pdiv(m, RW, inv_rw);
  j = m - t * RW;
  b = pdiv(t, RH, inv_rh);
  i = t - b * RH;
}

// epilogue flavour, a template parameter so each kernel holds only its own epilogue's registers
// (one generic epilogue - accumulate source + BN input/output quads + statistics live at once -
// needed ~250 VGPRs and spilled at 2 workgroups per CU)
enum { PW_EPI_PLAIN = 0, PW_EPI_STATS = 1, PW_EPI_ACC = 2, PW_EPI_BB = 3 };

template <int BM, int BN, int NS, int MINB, int EPI>
__global__ __launch_bounds__(PW_THREADS, MINB) void pw_kernel(const PwArgs a) {
  constexpr int WM = BM / 2, WN = BN / 2, TM = WM / 16, TN = WN / 16;
  constexpr int A_EL = BM * PW_BK, B_EL = BN * PW_BK, ST_EL = A_EL + B_EL;
  constexpr int NA = BM / 32, NB = BN / 32, P = NA + NB;  // 1-KB DMA pieces per thread and k-tile
  constexpr int SMEM_EL = pw_smem_el<BM, BN, NS>();
  __shared__ __attribute__((aligned(16))) bf16 smem[SMEM_EL];
  float* red = reinterpret_cast<float*>(smem + NS * ST_EL);

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w >> 1, wn = w & 1;
  const int tiles_n = a.N / BN;
  const int T = a.tiles_m * tiles_n;
  const int t_lo = (int)((long)T * blockIdx.x / gridDim.x), t_hi = (int)((long)T * (blockIdx.x + 1) / gridDim.x);
  const int cpt = a.SC / PW_BK;               // k-tiles per tap
  const int nk = a.ntaps * cpt;
  const int total = (t_hi - t_lo) * nk;
  const float inv_rw = 1.f / (float)a.RW, inv_rh = 1.f / (float)a.RH;
  // 1x1 / stride 1 / no offset: row m IS pixel m of the source (no decode, no mask)
  const bool direct = a.ntaps == 1 && a.dy[0] == 0 && a.dx[0] == 0 && a.istr == 1 && a.SH == a.RH && a.SW == a.RW;

  // ---- issue side: per piece the row's pixel base pointer and tap-validity mask of the tile being
  // streamed in (rows past M re-read row M-1: finite data whose results are neither stored nor counted)
  const int lrow = lane >> 3, lchunk = (lane & 7) ^ lrow;
  const bf16* a_row[NA];
  uint32_t a_mask[NA];
  const bf16* b_row[NB];
  const bf16* zpage = a.zeros + lchunk * 8;
  int i_ti = t_lo, i_tap = 0, i_cb = 0;
  auto set_rows = [&](int ti) {
    const int tm = ti / tiles_n, tn = ti - tm * tiles_n;
#pragma unroll
    for (int j = 0; j < NA; ++j) {
      const int m = min(tm * BM + (j * 4 + w) * 8 + lrow, a.M - 1);
      if (direct) {
        a_row[j] = a.A + (long)m * a.SC + lchunk * 8;
        a_mask[j] = 1u;
      } else {
        int b, i, jx;
        pw_rc(m, a.RH, a.RW, inv_rw, inv_rh, b, i, jx);
        const int iy = i * a.istr, ix = jx * a.istr;
        a_row[j] = a.A + (((long)b * a.SH + iy) * a.SW + ix) * a.SC + lchunk * 8;
        uint32_t mk = 0;
        for (int t = 0; t < a.ntaps; ++t) {
          const int sy = iy + a.dy[t], sx = ix + a.dx[t];
          mk |= ((unsigned)sy < (unsigned)a.SH && (unsigned)sx < (unsigned)a.SW) ? (1u << t) : 0u;
        }
        a_mask[j] = mk;
      }
    }
#pragma unroll
    for (int j = 0; j < NB; ++j) b_row[j] = a.W + (long)(tn * BN + (j * 4 + w) * 8 + lrow) * a.Ktot + lchunk * 8;
  };
  if (total > 0) set_rows(i_ti);
  auto issue = [&](int s) {  // k-tile (i_ti, i_tap, i_cb) = stream position s, then advance
    bf16* As = smem + (s % NS) * ST_EL;
    bf16* Bs = As + A_EL;
    const long toff = ((long)a.dy[i_tap] * a.SW + a.dx[i_tap]) * a.SC + i_cb * PW_BK;
    const int woff = a.kt[i_tap] * a.SC + i_cb * PW_BK;
#pragma unroll
    for (int j = 0; j < NA; ++j) glds16_async((a_mask[j] >> i_tap) & 1u ? a_row[j] + toff : zpage, As + (j * 4 + w) * 512);
#pragma unroll
    for (int j = 0; j < NB; ++j) glds16_async(b_row[j] + woff, Bs + (j * 4 + w) * 512);
    if (++i_cb == cpt) {
      i_cb = 0;
      if (++i_tap == a.ntaps) {
        i_tap = 0;
        if (++i_ti < t_hi) set_rows(i_ti);
      }
    }
  };

  f32x4_t acc[TN][TM];
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int i = 0; i < TM; ++i) acc[j][i] = f32x4_t{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (s < total) issue(s);

  int c_ti = t_lo, c_kt = 0;  // compute side
  int since_epi = 0;          // waits left that an epilogue's stores are younger than
  for (int s = 0; s < total; ++s) {
    // k-tile s has landed once at most the younger in-flight k-tiles are outstanding (over-waiting
    // near the stream's end and behind an epilogue's stores is harmless)
    // (vmcnt counts the epilogue's output stores too, and they are YOUNGER than the k-tiles issued
    // before them: for the NS-1 waits after an epilogue its TM*TN stores are allowed to stay in
    // flight - waiting for their write acknowledgements was most of this kernel's SQ_WAIT_ANY)
    if (s + NS - 2 >= total) {
      wait_vm<0>();
    } else if (since_epi > 0) {
      --since_epi;
      wait_vm<(NS - 2) * P + TM * TN>();
    } else {
      wait_vm<(NS - 2) * P>();
    }
    lds_barrier();  // every wave's DMA of k-tile s is visible; every wave is done reading k-tile s-1
    if (s + NS - 1 < total) issue(s + NS - 1);  // into k-tile s-1's stage

    const bf16* As = smem + (s % NS) * ST_EL;
    const bf16* Bs = As + A_EL;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int pc = (kk * 4 + (lane >> 4)) ^ (lane & 7);
      bf16x8_t af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i)
        af[i] = *reinterpret_cast<const bf16x8_t*>(As + (wm * WM + i * 16 + (lane & 15)) * PW_BK + pc * 8);
#pragma unroll
      for (int j = 0; j < TN; ++j)
        bfr[j] = *reinterpret_cast<const bf16x8_t*>(Bs + (wn * WN + j * 16 + (lane & 15)) * PW_BK + pc * 8);
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int i = 0; i < TM; ++i)
          acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[j][i], 0, 0, 0);
    }

    if (++c_kt < nk) continue;
    c_kt = 0;
    // ---------------------------------------------------------------- epilogue of tile c_ti
    const int tm = c_ti / tiles_n, tn = c_ti - tm * tiles_n;
    ++c_ti;
    const int m0 = tm * BM + wm * WM;                       // this wave's first row
    const int n0 = tn * BN + wn * WN + 4 * (lane >> 4);     // + 16 j + q: this lane's channels
    // lane holds D[n][m]: channels n0 + 16j + q (q = 0..3), pixel m0 + 16i + (lane & 15)
    bf16* orow[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int m = m0 + i * 16 + (lane & 15);
      long pix = m;
      if (!direct || a.ostr != 1) {
        int b, ii, jx;
        pw_rc(m, a.RH, a.RW, inv_rw, inv_rh, b, ii, jx);
        pix = ((long)b * a.OHf + ii * a.ostr + a.oy) * a.OWf + jx * a.ostr + a.ox;
      }
      orow[i] = m < a.M ? a.out + pix * a.N + n0 : nullptr;
      // rows past M store into the sink page: every lane issues exactly TM*TN stores, the count the
      // waits above rely on (a branch around a store would make it smaller)
    }
    // epilogue operands, every load before the first use (one latency, not TM*TN): the old
    // output (accumulate) and, for the data gradient's BatchNorm-backward statistics, the BN's input
    // x (and its output y for a mask that cannot be recomputed from x) at the same positions
    constexpr bool bb = EPI == PW_EPI_BB;
    const bool bb_from_x = bb && a.bb_y == nullptr && a.bb_act == ACT_RELU;
    const bool bb_need_y = bb && a.bb_act != ACT_NONE && !bb_from_x;
    u32x2_t old[TN][TM], xv[TN][TM], yv[TN][TM];
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const long off = orow[i] ? (long)(orow[i] - a.out) + 16 * j : 0;
        if (EPI == PW_EPI_ACC) old[j][i] = orow[i] ? *reinterpret_cast<const u32x2_t*>(a.out + off) : u32x2_t{0u, 0u};
        if (bb) xv[j][i] = *reinterpret_cast<const u32x2_t*>(a.bb_x + off);
        if (bb_need_y) yv[j][i] = *reinterpret_cast<const u32x2_t*>(a.bb_y + off);
      }
    float ssum[TN][4], ssq[TN][4], kshift[TN][4];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      float bmean[4], binv[4], bsc[4], bsh[4];
      if (bb) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int c = n0 + 16 * j + q;
          bmean[q] = a.bb_mean[c];
          binv[q] = a.bb_invstd[c];
          if (bb_from_x) {  // = norm.hip BwdMask: bit-identical to the forward's pre-activation
            bsc[q] = a.bb_gamma[c] * binv[q];
            bsh[q] = a.bb_beta[c] - bmean[q] * bsc[q];
          }
          ssum[j][q] = ssq[j][q] = 0.f;
          kshift[j][q] = 0.f;
        }
      }
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        f32x4_t v = acc[j][i];
        if (EPI == PW_EPI_ACC) {
          v[0] += bf2f((bf16)(old[j][i][0] & 0xffffu)); v[1] += bf2f((bf16)(old[j][i][0] >> 16));
          v[2] += bf2f((bf16)(old[j][i][1] & 0xffffu)); v[3] += bf2f((bf16)(old[j][i][1] >> 16));
        }
        const u32x2_t pk = {pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3])};
        *reinterpret_cast<u32x2_t*>(orow[i] ? orow[i] + 16 * j : a.sink + ((n0 + 16 * j) & 8191)) = pk;
        acc[j][i] = f32x4_t{0.f, 0.f, 0.f, 0.f};
        const float y[4] = {bf2f((bf16)(pk[0] & 0xffffu)), bf2f((bf16)(pk[0] >> 16)), bf2f((bf16)(pk[1] & 0xffffu)),
                            bf2f((bf16)(pk[1] >> 16))};
        const bool ok = orow[i] != nullptr;
        if (bb) {
          // BatchNorm-backward statistics of the stored (final) values: g = out * act'(.)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const uint32_t xw = xv[j][i][q >> 1] >> (16 * (q & 1));
            const float x = bf2f((bf16)(xw & 0xffffu));
            float g = y[q];
            if (bb_from_x) {
              g = (x * bsc[q] + bsh[q]) > 0.f ? g : 0.f;
            } else if (bb_need_y) {
              g *= act_grad_from_out(bf2f((bf16)((yv[j][i][q >> 1] >> (16 * (q & 1))) & 0xffffu)), a.bb_act);
            }
            g = ok ? g : 0.f;
            ssum[j][q] += g;
            ssq[j][q] += g * (x - bmean[q]) * binv[q];
          }
        } else if (EPI == PW_EPI_STATS) {
          // forward statistics of the STORED values, shifted by the wave's first row (numerically safe)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            if (i == 0) {
              kshift[j][q] = __shfl(y[q], lane & 48, 64);
              ssum[j][q] = ssq[j][q] = 0.f;
            }
            const float d = ok ? y[q] - kshift[j][q] : 0.f;
            ssum[j][q] += d;
            ssq[j][q] += d * d;
          }
        }
      }
    }
    since_epi = NS - 1;
    if (EPI != PW_EPI_STATS && EPI != PW_EPI_BB) continue;
    // reduce over the 16 pixels of a lane group, then fold the two wave rows (fixed order)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
          ssum[j][q] += __shfl_xor(ssum[j][q], o, 64);
          ssq[j][q] += __shfl_xor(ssq[j][q], o, 64);
        }
      }
    if ((lane & 15) == 0) {
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int c = wn * WN + 16 * j + 4 * (lane >> 4) + q;
          float* r = red + (wm * BN + c) * 4;
          r[0] = kshift[j][q];
          r[1] = ssum[j][q];
          r[2] = ssq[j][q];
        }
    }
    lds_barrier();
    if (tid < BN) {
      const int c = tid;
      const float* r0 = red + c * 4;
      const float* r1 = red + (BN + c) * 4;
      const float K0 = r0[0];
      float S = r0[1], Q = r0[2];
      const int n1 = min(WM, a.M - (tm * BM + WM));
      if (n1 > 0) {
        const float d = r1[0] - K0;
        S += r1[1] + n1 * d;
        Q += r1[2] + 2.f * d * r1[1] + n1 * d * d;
      }
      float* pp = a.bn_part + (long)tm * 3 * a.N + tn * BN + c;
      pp[0] = K0;
      pp[a.N] = S;
      pp[2 * a.N] = Q;
    }
    // (the next write of `red` is a full k-loop iteration - and its barrier - away)
  }
}

// DTFE_PW="<mode>[,cfg=<id>][,grid=<workgroups>][,mintiles=<n>]" (A/B and tests): mode off | bb |
// all, see run_igemm_pipe; the options override the tile / ring choice, the grid and the
// smallest launch that goes persistent.
int pw_opt(const char* key, int dflt) {
  const char* e = std::getenv("DTFE_PW");
  const size_t n = std::strlen(key);
  while (e && *e) {
    if (!std::strncmp(e, key, n) && e[n] == '=') return std::atoi(e + n + 1);
    e = std::strchr(e, ',');
    if (e) ++e;
  }
  return dflt;
}

enum { PW_MODE_OFF = 0, PW_MODE_BB = 1, PW_MODE_ALL = 2 };
int pw_mode() {
  const char* e = std::getenv("DTFE_PW");
  if (!e || !*e) return PW_DEFAULT_MODE;
  if (!std::strncmp(e, "off", 3)) return PW_MODE_OFF;
  if (!std::strncmp(e, "bb", 2)) return PW_MODE_BB;
  return PW_MODE_ALL;
}

template <int BM, int BN, int NS, int MINB>
void launch_pw(PwArgs& a, int epi, hipStream_t s) {
  a.tiles_m = (a.M + BM - 1) / BM;
  const int T = a.tiles_m * (a.N / BN);
  int grid = 256 * MINB;
  const int g_env = pw_opt("grid", 0);
  if (g_env > 0) grid = g_env;
  grid = std::min(grid, T);
  switch (epi) {
    case PW_EPI_STATS: hipLaunchKernelGGL((pw_kernel<BM, BN, NS, MINB, PW_EPI_STATS>), dim3(grid), dim3(PW_THREADS), 0, s, a); break;
    case PW_EPI_ACC: hipLaunchKernelGGL((pw_kernel<BM, BN, NS, MINB, PW_EPI_ACC>), dim3(grid), dim3(PW_THREADS), 0, s, a); break;
    case PW_EPI_BB: hipLaunchKernelGGL((pw_kernel<BM, BN, NS, MINB, PW_EPI_BB>), dim3(grid), dim3(PW_THREADS), 0, s, a); break;
    default: hipLaunchKernelGGL((pw_kernel<BM, BN, NS, MINB, PW_EPI_PLAIN>), dim3(grid), dim3(PW_THREADS), 0, s, a); break;
  }
}

// tile / ring choice (DTFE_PW cfg=<id> for A/B): 0 = 128x128 NS2 (2 WG/CU), 1 = 128x128 NS3 (1 WG/CU),
// 2 = 128x64 NS3 (2 WG/CU), 3 = 128x128 NS4 (1 WG/CU)
int pw_cfg(int N) {
  const int e = pw_opt("cfg", -1);
  if (e >= 0 && e <= 3 && (e == 2 || N % 128 == 0)) return e;
  return N % 128 == 0 ? 0 : 2;
}

void run_pw(PwArgs& a, int epi, hipStream_t s) {
  switch (pw_cfg(a.N)) {
    case 1: launch_pw<128, 128, 3, 1>(a, epi, s); break;
    case 2: launch_pw<128, 64, 3, 2>(a, epi, s); break;
    case 3: launch_pw<128, 128, 4, 1>(a, epi, s); break;
    default: launch_pw<128, 128, 2, 2>(a, epi, s); break;
  }
}

}  // namespace

bool run_igemm_pipe(const IgemmArgs& g, long Mmax, hipStream_t s) {
  const int mode = pw_mode();
  if (mode == PW_MODE_OFF || (mode == PW_MODE_BB && !g.bb_x) || g.nphase != 1 || g.SC % PW_BK || g.N % 64) return false;
  const IgPhase& P = g.ph[0];
  if (P.ntaps < 1) return false;
  PwArgs a;
  std::memset(&a, 0, sizeof(a));
  a.A = g.src; a.W = g.w; a.out = g.out; a.zeros = g.zeros; a.sink = ig_sink_page(s);
  a.M = (int)Mmax; a.N = g.N; a.SC = g.SC; a.Ktot = g.Ktot;
  a.RH = P.RH; a.RW = P.RW; a.SH = g.SH; a.SW = g.SW; a.istr = g.istr;
  a.OHf = g.OHf; a.OWf = g.OWf; a.ostr = g.ostr; a.oy = P.oy; a.ox = P.ox;
  a.ntaps = P.ntaps;
  for (int t = 0; t < P.ntaps; ++t) { a.dy[t] = P.dy[t]; a.dx[t] = P.dx[t]; a.kt[t] = P.kt[t]; }
  a.accum = g.accum;
  a.bn_part = g.bn_part;
  if (g.bb_x) {
    a.bb_x = g.bb_x; a.bb_y = g.bb_y; a.bb_mean = g.bb_mean; a.bb_invstd = g.bb_invstd;
    a.bb_gamma = g.bb_gamma; a.bb_beta = g.bb_beta; a.bb_act = g.bb_act;
  }
  // one epilogue flavour per launch (the combinations no conv issues stay on the per-tile kernel)
  const int epi = g.bb_x ? PW_EPI_BB : g.bn_part ? PW_EPI_STATS : g.accum ? PW_EPI_ACC : PW_EPI_PLAIN;
  if ((g.bb_x || g.bn_part) && g.accum) return false;
  if (g.acc_src) return false;  // (the masked accumulation source: per-tile kernel only)
  // too few tiles for a persistent grid: the per-tile kernel's split-K spreads them better
  const int bn = pw_cfg(a.N) == 2 ? 64 : 128;
  const long tiles = (Mmax + 127) / 128 * (a.N / bn);
  const long min_tiles = pw_opt("mintiles", 256);
  if (tiles < min_tiles) return false;
  run_pw(a, epi, s);
  return true;
}

}  // namespace dtfe
