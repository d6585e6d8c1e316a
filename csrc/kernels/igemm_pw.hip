// Pointwise (1x1) convolutions as persistent, pipelined GEMMs on gfx950 - the 1x1 convs are two
// thirds of ResNet-50's conv time (profiles/r3_resnet50_convs_b256.txt: 8.3 of 12.9 ms).
//
//   forward   Y[m][n] = sum_c X[pix(m)][c] W[n][c]         (stride 1: pix(m) = m; stride 2: the
//             strided source pixel) + BatchNorm statistics of the stored bf16 Y per tile
//   dgrad     dX[pix(m)][c] (+)= sum_n dY[m][n] Wt[c][n]   (stride 2 only accumulating: the three
//             other parity phases of dX get nothing and keep the shortcut's share)
//
// Against the per-tile implicit-GEMM kernel (igemm.hip) this launch
//   * is persistent: one (or two) workgroups per CU walk a contiguous run of output tiles, and the
//     k-tile stream runs ACROSS tile boundaries - the next tile's first k-tiles are in flight while
//     the current tile's epilogue runs (the 1x1 layers have 1-16 k-tiles per tile, so the per-tile
//     load latency and epilogue were most of their time);
//   * keeps NS-1 k-tiles in flight: an NS-stage LDS ring filled by global_load_lds_dwordx4, counted
//     `s_waitcnt vmcnt(N)` and raw s_barrier (no vmcnt(0) drain per k-tile);
//   * has no per-k-tile address math: each row's base pointer is computed once per tile (the
//     1x1 row is one pixel), a k-tile is a +128 B step;
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
constexpr int PW_BK = 64;

typedef __attribute__((address_space(3))) void lds_void_t;

__device__ __forceinline__ void glds16(const void* g, bf16* lds_piece) {
  __builtin_amdgcn_global_load_lds(g, (lds_void_t*)lds_piece, 16, 0, 0);
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

// pixel index of GEMM row m on a (RH x RW) grid with stride `str` into a (SH x SW) image
__device__ __forceinline__ long pw_pix(int m, int str, int RH, int RW, int SH, int SW, float inv_rw, float inv_rh) {
  if (str == 1) return m;
  const int t = pdiv(m, RW, inv_rw), j = m - t * RW;
  const int b = pdiv(t, RH, inv_rh), i = t - b * RH;
  return ((long)b * SH + i * str) * SW + j * str;
}

template <int BM, int BN, int NS, int MINB>
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
  const int nk = a.K / PW_BK;
  const int total = (t_hi - t_lo) * nk;
  const float inv_rw = 1.f / (float)a.RW, inv_rh = 1.f / (float)a.RH;

  // ---- issue side: row pointers of the tile being streamed in (rows past M re-read row M-1:
  // finite data whose results are neither stored nor counted)
  const int lrow = lane >> 3, lchunk = (lane & 7) ^ lrow;
  const bf16* a_row[NA];
  const bf16* b_row[NB];
  int i_ti = t_lo, i_kt = 0;
  auto set_rows = [&](int ti) {
    const int tm = ti / tiles_n, tn = ti - tm * tiles_n;
#pragma unroll
    for (int j = 0; j < NA; ++j) {
      const int m = min(tm * BM + (j * 4 + w) * 8 + lrow, a.M - 1);
      a_row[j] = a.A + pw_pix(m, a.istr, a.RH, a.RW, a.SH, a.SW, inv_rw, inv_rh) * a.K + lchunk * 8;
    }
#pragma unroll
    for (int j = 0; j < NB; ++j) b_row[j] = a.W + (long)(tn * BN + (j * 4 + w) * 8 + lrow) * a.K + lchunk * 8;
  };
  if (total > 0) set_rows(i_ti);
  auto issue = [&](int s) {  // k-tile (i_ti, i_kt) = stream position s, then advance
    bf16* As = smem + (s % NS) * ST_EL;
    bf16* Bs = As + A_EL;
#pragma unroll
    for (int j = 0; j < NA; ++j) glds16(a_row[j] + i_kt * PW_BK, As + (j * 4 + w) * 512);
#pragma unroll
    for (int j = 0; j < NB; ++j) glds16(b_row[j] + i_kt * PW_BK, Bs + (j * 4 + w) * 512);
    if (++i_kt == nk) {
      i_kt = 0;
      if (++i_ti < t_hi) set_rows(i_ti);
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
  for (int s = 0; s < total; ++s) {
    // k-tile s has landed once at most the younger in-flight k-tiles are outstanding (over-waiting
    // near the stream's end and behind an epilogue's stores is harmless)
    if (s + NS - 2 < total) wait_vm<(NS - 2) * P>();
    else wait_vm<0>();
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
      orow[i] = m < a.M ? a.out + pw_pix(m, a.ostr, a.RH, a.RW, a.OHf, a.OWf, inv_rw, inv_rh) * a.N + n0 : nullptr;
    }
    u32x2_t old[TN][TM];
    if (a.accum) {  // every load before the first add (one latency, not TM*TN)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int i = 0; i < TM; ++i)
          old[j][i] = orow[i] ? *reinterpret_cast<const u32x2_t*>(orow[i] + 16 * j) : u32x2_t{0u, 0u};
    }
    float ssum[TN][4], ssq[TN][4], kshift[TN][4];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        f32x4_t v = acc[j][i];
        if (a.accum) {
          v[0] += bf2f((bf16)(old[j][i][0] & 0xffffu)); v[1] += bf2f((bf16)(old[j][i][0] >> 16));
          v[2] += bf2f((bf16)(old[j][i][1] & 0xffffu)); v[3] += bf2f((bf16)(old[j][i][1] >> 16));
        }
        const u32x2_t pk = {pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3])};
        if (orow[i]) *reinterpret_cast<u32x2_t*>(orow[i] + 16 * j) = pk;
        acc[j][i] = f32x4_t{0.f, 0.f, 0.f, 0.f};
        if (a.bn_part) {
          // statistics of the STORED values, shifted by the wave's first row (numerically safe)
          const float y[4] = {bf2f((bf16)(pk[0] & 0xffffu)), bf2f((bf16)(pk[0] >> 16)), bf2f((bf16)(pk[1] & 0xffffu)),
                              bf2f((bf16)(pk[1] >> 16))};
          const bool ok = orow[i] != nullptr;
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
    if (!a.bn_part) continue;
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

int env_int(const char* name, int dflt) {
  const char* v = std::getenv(name);
  return v && *v ? std::atoi(v) : dflt;
}

template <int BM, int BN, int NS, int MINB>
void launch_pw(PwArgs& a, hipStream_t s) {
  a.tiles_m = (a.M + BM - 1) / BM;
  const int T = a.tiles_m * (a.N / BN);
  int grid = 256 * MINB;
  const int g_env = env_int("DTFE_PW_GRID", 0);
  if (g_env > 0) grid = g_env;
  grid = std::min(grid, T);
  hipLaunchKernelGGL((pw_kernel<BM, BN, NS, MINB>), dim3(grid), dim3(PW_THREADS), 0, s, a);
}

// tile / ring choice (DTFE_PW_CFG=<id> for A/B): 0 = 128x128 NS2 (2 WG/CU), 1 = 128x128 NS3 (1 WG/CU),
// 2 = 128x64 NS3 (2 WG/CU), 3 = 128x128 NS4 (1 WG/CU)
int pw_cfg(int N) {
  const int e = env_int("DTFE_PW_CFG", -1);
  if (e >= 0 && e <= 3 && (e == 2 || N % 128 == 0)) return e;
  return N % 128 == 0 ? 0 : 2;
}

void run_pw(PwArgs& a, hipStream_t s) {
  switch (pw_cfg(a.N)) {
    case 1: launch_pw<128, 128, 3, 1>(a, s); break;
    case 2: launch_pw<128, 64, 3, 2>(a, s); break;
    case 3: launch_pw<128, 128, 4, 1>(a, s); break;
    default: launch_pw<128, 128, 2, 2>(a, s); break;
  }
}

}  // namespace

bool launch_pw_fwd(const ConvFwdArgs& f, hipStream_t s, bool* stats_done) {
  const ConvGeom& g = f.g;
  if (g.KH != 1 || g.KW != 1 || g.pad != 0 || g.C % PW_BK || g.Cout % 64 || g.pool_order || f.bias || f.act != 0)
    return false;
  if (env_int("DTFE_PW_OFF", 0)) return false;
  PwArgs a;
  std::memset(&a, 0, sizeof(a));
  a.A = f.x; a.W = f.w; a.out = f.y;
  a.M = g.B * g.OH * g.OW; a.N = g.Cout; a.K = g.C;
  a.RH = g.OH; a.RW = g.OW; a.SH = g.H; a.SW = g.W; a.istr = g.stride;
  a.OHf = g.OH; a.OWf = g.OW; a.ostr = 1;
  const int tiles_m = (a.M + 127) / 128;
  if (f.bn_stats) a.bn_part = bn_part_buffer(tiles_m, a.N, s);
  run_pw(a, s);
  if (f.bn_stats) launch_bn_part_reduce(a.bn_part, tiles_m, a.N, a.M, 128, f.bn_stats, s);
  if (stats_done) *stats_done = f.bn_stats != nullptr;
  return true;
}

bool launch_pw_dgrad(const ConvDgradArgs& d, hipStream_t s) {
  const ConvGeom& g = d.g;
  if (g.KH != 1 || g.KW != 1 || g.pad != 0 || g.Cout % PW_BK || g.C % 64 || d.unpool || d.relu_mask || d.bnb_stats)
    return false;
  if (g.stride != 1 && !(g.stride == 2 && d.accumulate)) return false;
  if (env_int("DTFE_PW_OFF", 0)) return false;
  PwArgs a;
  std::memset(&a, 0, sizeof(a));
  a.A = d.dy; a.W = d.wt; a.out = d.dx;
  a.M = g.B * g.OH * g.OW; a.N = g.C; a.K = g.Cout;
  a.RH = g.OH; a.RW = g.OW; a.SH = g.OH; a.SW = g.OW; a.istr = 1;
  a.OHf = g.H; a.OWf = g.W; a.ostr = g.stride;
  a.accum = d.accumulate;
  run_pw(a, s);
  return true;
}

}  // namespace dtfe
