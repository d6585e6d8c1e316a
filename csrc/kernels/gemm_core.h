// Generic LDS-tiled MFMA GEMM engine for gfx950.
//
//   C[m][n] = sum_k  A(m,k) * B(n,k)        (then an epilogue functor)
//
// Both operands are described by a *loader*: a policy object that moves one
// BK-deep k-tile of its operand from global memory into LDS through registers
// (register staging, double-buffered LDS, one barrier per k-tile: the
// "minimum 2-phase" structure of the CDNA HIP guide, STAGE issued before the
// MFMAs of the current tile, LDS write after them).  The LDS image a loader
// writes depends on the global layout of its operand:
//
//   KMAJ  (k contiguous in global):    LDS [rows][BK+pad], fragments by ds_read_b128
//   RMAJ  (rows contiguous in global): bf16 -> LDS [BK][SR] read with the gfx950
//                                      ds_read_b64_tr_b16 transpose (2 per fragment)
//                                      f32  -> transposed while staging into [rows][BK+pad]
//
// The k order inside a 16x16x32 bf16 fragment is the natural one; for f32
// (v_mfma_f32_16x16x4_f32, exact fp32) each lane reads a float4 of k and feeds
// its 4 elements to 4 consecutive MFMAs - a k permutation applied identically
// to both operands, so the dot product is unchanged.
#pragma once
#include "common.h"

namespace dtfe {

constexpr int GEMM_THREADS = 256;  // 4 waves
constexpr int BK = 32;             // default k-tile depth (conv loaders); dense GEMMs use 64

enum Mode : int { KMAJ = 0, RMAJ = 1 };

template <typename T> struct ElemT;
template <> struct ElemT<bf16> { static constexpr int VEC = 8; };
template <> struct ElemT<float> { static constexpr int VEC = 4; };

// ---------------------------------------------------------------- LDS layout
template <typename T, int R, int MODE, int KB = BK> struct LdsLayout;

// KMAJ image: [R][KB + PADK].  Rows are 16*(odd) bytes (bf16 80/144 B, f32
// 144/272 B): the 16 lanes reading 16 distinct rows at one k-chunk hit 16
// distinct 4-bank groups.
template <typename T, int R, int KB> struct LdsLayout<T, R, KMAJ, KB> {
  static constexpr int PADK = 16 / sizeof(T);
  static constexpr int LD = KB + PADK;
  static constexpr int ELEMS = R * LD;
};
// f32 RMAJ operands are transposed during staging into the KMAJ image.
template <int R, int KB> struct LdsLayout<float, R, RMAJ, KB> : LdsLayout<float, R, KMAJ, KB> {};
// bf16 RMAJ image: [BK][SR] with SR*2 bytes == 64 (mod 128) and the columns of
// rows with bit 3 set XOR-ed by 16 elements (32 B): the 8 rows one 32-lane half
// touches in a ds_read_b64_tr_b16 then cover the 64 banks exactly once.
template <int R, int KB> struct LdsLayout<bf16, R, RMAJ, KB> {
  static constexpr int SR = ((2 * R) % 128 == 64) ? R : R + 32;
  static constexpr int LD = SR;
  static constexpr int ELEMS = KB * SR;
  static __device__ __forceinline__ int off(int k, int c) { return k * SR + (c ^ (((k >> 3) & 1) << 4)); }
};

// ------------------------------------------------------------------ staging
// Chunk enumeration shared by all loaders: a k-tile of an R-row operand is
// R*BK/VEC 16-byte chunks.  KMAJ: chunk idx -> (r = idx / (BK/VEC), k = idx % (BK/VEC) * VEC)
// RMAJ: idx -> (k = idx / (R/VEC), r = idx % (R/VEC) * VEC).
template <typename T, int R, int MODE, int KB = BK>
struct Chunks {
  static constexpr int VEC = ElemT<T>::VEC;
  static constexpr int N = R * KB / VEC;
  static constexpr int NC = (N + GEMM_THREADS - 1) / GEMM_THREADS;
  static __device__ __forceinline__ void rk(int idx, int& r, int& k) {
    if constexpr (MODE == KMAJ) { r = idx / (KB / VEC); k = (idx % (KB / VEC)) * VEC; }
    else { k = idx / (R / VEC); r = (idx % (R / VEC)) * VEC; }
  }
};

template <typename T, int R, int MODE, int KB = BK>
__device__ __forceinline__ void stage_store(T* lds, const u32x4_t* rg) {
  using Lay = LdsLayout<T, R, MODE, KB>;
  using C = Chunks<T, R, MODE, KB>;
  const int tid = threadIdx.x;
#pragma unroll
  for (int c = 0; c < C::NC; ++c) {
    const int idx = tid + c * GEMM_THREADS;
    if (C::N % GEMM_THREADS == 0 || idx < C::N) {
      int r, k;
      C::rk(idx, r, k);
      if constexpr (MODE == KMAJ) {
        *reinterpret_cast<u32x4_t*>(lds + r * Lay::LD + k) = rg[c];
      } else if constexpr (sizeof(T) == 2) {
        *reinterpret_cast<u32x4_t*>(lds + Lay::off(k, r)) = rg[c];
      } else {
        const float* e = reinterpret_cast<const float*>(&rg[c]);
#pragma unroll
        for (int i = 0; i < C::VEC; ++i) lds[(r + i) * Lay::LD + k] = e[i];
      }
    }
  }
}

template <typename T> __device__ __forceinline__ T one_val() {
  if constexpr (sizeof(T) == 2) return (T)0x3f80; else return (T)1.0f;
}

// Dense operand: element (r, k) of a rows x K matrix.
//   KMAJ: p[r*ld + k]      RMAJ: p[k*ld + r]
// ones_row >= 0 makes row `ones_row` read as 1.0 for every k < K (the bias
// column of the weight-gradient GEMMs).
template <typename T, int R, int MODE, int KB = BK>
struct DenseLoader {
  using Lay = LdsLayout<T, R, MODE, KB>;
  using C = Chunks<T, R, MODE, KB>;
  static constexpr int VEC = C::VEC;

  const T* p; long ld; int rows; int K; int r0; int ones_row; bool vec_ok, rows_full;
  const T* base[C::NC];  // this thread's chunk addresses at k0 = 0
  u32x4_t regs[C::NC];

  __device__ __forceinline__ DenseLoader(const T* p_, long ld_, int rows_, int K_, int r0_, int ones_row_ = -1)
      : p(p_), ld(ld_), rows(rows_), K(K_), r0(r0_), ones_row(ones_row_) {
    vec_ok = ((ld % VEC) == 0) && ((((uintptr_t)p) & 15) == 0);
    // block-uniform: every row of this tile exists, no ones row inside, 16 B aligned
    rows_full = vec_ok && r0 + R <= rows && !(ones_row >= r0 && ones_row < r0 + R);
#pragma unroll
    for (int c = 0; c < C::NC; ++c) {
      int r, k;
      C::rk(threadIdx.x + c * GEMM_THREADS, r, k);
      base[c] = MODE == KMAJ ? p + (long)(r0 + r) * ld + k : p + (long)k * ld + r0 + r;
    }
  }

  // FAST: the caller guarantees an interior tile (rows_full, k0 + KB <= K)
  template <bool FAST = false>
  __device__ __forceinline__ void load(int k0) {
    if (FAST || (rows_full && k0 + KB <= K)) {
      // interior tile: branch-free 16 B loads, all in flight together
      const long step = MODE == KMAJ ? (long)k0 : (long)k0 * ld;
#pragma unroll
      for (int c = 0; c < C::NC; ++c)
        if (C::N % GEMM_THREADS == 0 || threadIdx.x + c * GEMM_THREADS < C::N)
          regs[c] = *reinterpret_cast<const u32x4_t*>(base[c] + step);
      return;
    }
    const int tid = threadIdx.x;
#pragma unroll
    for (int c = 0; c < C::NC; ++c) {
      const int idx = tid + c * GEMM_THREADS;
      u32x4_t v = {0u, 0u, 0u, 0u};
      if (C::N % GEMM_THREADS == 0 || idx < C::N) {
        int r, k;
        C::rk(idx, r, k);
        const int gr = r0 + r, gk = k0 + k;
        T* e = reinterpret_cast<T*>(&v);
        if constexpr (MODE == KMAJ) {
          if (gr < rows) {
            if (gr == ones_row) {
#pragma unroll
              for (int i = 0; i < VEC; ++i) if (gk + i < K) e[i] = one_val<T>();
            } else if (vec_ok && gk + VEC <= K) {
              v = *reinterpret_cast<const u32x4_t*>(p + (long)gr * ld + gk);
            } else {
#pragma unroll
              for (int i = 0; i < VEC; ++i) if (gk + i < K) e[i] = p[(long)gr * ld + gk + i];
            }
          }
        } else {
          if (gk < K) {
            const bool has_one = ones_row >= gr && ones_row < gr + VEC;
            if (vec_ok && gr + VEC <= rows && !has_one) {
              v = *reinterpret_cast<const u32x4_t*>(p + (long)gk * ld + gr);
            } else {
#pragma unroll
              for (int i = 0; i < VEC; ++i) {
                if (gr + i == ones_row) e[i] = one_val<T>();
                else if (gr + i < rows) e[i] = p[(long)gk * ld + gr + i];
              }
            }
          }
        }
      }
      regs[c] = v;
    }
  }
  __device__ __forceinline__ void store(T* lds) const { stage_store<T, R, MODE, KB>(lds, regs); }
  // interior-tile load into a caller-owned register set (the deep-prefetch k-loop's ring)
  __device__ __forceinline__ void load_into(int k0, u32x4_t (&r)[C::NC]) const {
    const long step = MODE == KMAJ ? (long)k0 : (long)k0 * ld;
#pragma unroll
    for (int c = 0; c < C::NC; ++c)
      if (C::N % GEMM_THREADS == 0 || threadIdx.x + c * GEMM_THREADS < C::N)
        r[c] = *reinterpret_cast<const u32x4_t*>(base[c] + step);
  }
  __device__ __forceinline__ void store_from(T* lds, const u32x4_t (&r)[C::NC]) const {
    stage_store<T, R, MODE, KB>(lds, r);
  }
  // every k-tile of [k_begin, k_end) is interior (block-uniform)
  __device__ __forceinline__ bool all_fast(int k_begin, int k_end) const {
    return rows_full && (k_end - k_begin) % KB == 0 && k_end <= K;
  }
};

// loaders that provide all_fast()/load<FAST> (conv loaders take the generic loop)
template <typename L, typename = void> struct requires_fast_check { static constexpr bool value = false; };
template <typename L>
struct requires_fast_check<L, decltype((void)&L::all_fast)> { static constexpr bool value = true; };

// ---------------------------------------------------------------- tile config
template <typename T, int BM_, int BN_, int WARPS_M_, int WARPS_N_, int BK_ = BK>
struct TileCfg {
  static_assert(WARPS_M_ * WARPS_N_ == 4, "4 waves per workgroup");
  static_assert(BK_ % 32 == 0, "k-tile is a multiple of the 32-deep bf16 MFMA");
  static constexpr int BM = BM_, BN = BN_, WARPS_M = WARPS_M_, WARPS_N = WARPS_N_, BK = BK_;
  static constexpr int WM = BM / WARPS_M, WN = BN / WARPS_N;
  static constexpr int TM = WM / 16, TN = WN / 16;
  static constexpr int WAVES = 4;  // waves holding the accumulators (dense_epilogue)
  static_assert(TM >= 1 && TN >= 1, "wave tile must be >= 16x16");
};

// ------------------------------------------------------------- MFMA compute
template <int R, int MODE, int KB = BK>
__device__ __forceinline__ bf16x8_t frag_bf16(const bf16* lds, int rbase, int kk, int lane) {
  if constexpr (MODE == KMAJ) {
    using L = LdsLayout<bf16, R, KMAJ, KB>;
    return *reinterpret_cast<const bf16x8_t*>(lds + (rbase + (lane & 15)) * L::LD + kk + 8 * (lane >> 4));
  } else {
    using L = LdsLayout<bf16, R, RMAJ, KB>;
    const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
    const int c = rbase + 4 * p;
    s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4_t, lds + L::off(kk + 8 * g + q, c)));
    s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4_t, lds + L::off(kk + 8 * g + 4 + q, c)));
    s16x8_t v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8_t, v);
  }
}

template <int R, int KB = BK>
__device__ __forceinline__ f32x4_t frag_f32(const float* lds, int rbase, int h, int lane) {
  using L = LdsLayout<float, R, KMAJ, KB>;
  return *reinterpret_cast<const f32x4_t*>(lds + (rbase + (lane & 15)) * L::LD + 16 * h + 4 * (lane >> 4));
}

template <typename T, typename Cfg, int AMODE, int BMODE>
__device__ __forceinline__ void tile_compute(const T* As, const T* Bs, int wm, int wn, int lane,
                                             f32x4_t (&acc)[Cfg::TM][Cfg::TN]) {
  constexpr int KB = Cfg::BK;
  if constexpr (sizeof(T) == 2) {
#pragma unroll
    for (int kk = 0; kk < KB; kk += 32) {
      bf16x8_t a[Cfg::TM], b[Cfg::TN];
#pragma unroll
      for (int i = 0; i < Cfg::TM; ++i) a[i] = frag_bf16<Cfg::BM, AMODE, KB>(As, wm * Cfg::WM + i * 16, kk, lane);
#pragma unroll
      for (int j = 0; j < Cfg::TN; ++j) b[j] = frag_bf16<Cfg::BN, BMODE, KB>(Bs, wn * Cfg::WN + j * 16, kk, lane);
#pragma unroll
      for (int i = 0; i < Cfg::TM; ++i)
#pragma unroll
        for (int j = 0; j < Cfg::TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
  } else {
#pragma unroll
    for (int h = 0; h < KB / 16; ++h) {
      f32x4_t a[Cfg::TM], b[Cfg::TN];
#pragma unroll
      for (int i = 0; i < Cfg::TM; ++i) a[i] = frag_f32<Cfg::BM, KB>(As, wm * Cfg::WM + i * 16, h, lane);
#pragma unroll
      for (int j = 0; j < Cfg::TN; ++j) b[j] = frag_f32<Cfg::BN, KB>(Bs, wn * Cfg::WN + j * 16, h, lane);
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int i = 0; i < Cfg::TM; ++i)
#pragma unroll
          for (int j = 0; j < Cfg::TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i][s], b[j][s], acc[i][j], 0, 0, 0);
    }
  }
}

template <typename T, typename Cfg, typename LA, typename LB>
struct SmemSize {
  static constexpr int ELEMS = 2 * LA::Lay::ELEMS + 2 * LB::Lay::ELEMS;
  static constexpr int BYTES = ELEMS * sizeof(T);
};

// Runs the k-loop over [k_begin, k_end) and leaves the result in acc.
// Accumulator (i, j) of wave (wm, wn) covers rows wm*WM + i*16 + (lane>>4)*4 + 0..3
// and column wn*WN + j*16 + (lane&15) of the block tile.
template <bool FAST, typename T, typename Cfg, int AMODE, int BMODE, typename LA, typename LB>
__device__ __forceinline__ void gemm_kloop(LA& la, LB& lb, int k_begin, int nk, T* smem,
                                           f32x4_t (&acc)[Cfg::TM][Cfg::TN]) {
  constexpr int KB = Cfg::BK;
  constexpr int A_ELEMS = LA::Lay::ELEMS, B_ELEMS = LB::Lay::ELEMS;
  T* As0 = smem;
  T* As1 = smem + A_ELEMS;
  T* Bs0 = smem + 2 * A_ELEMS;
  T* Bs1 = smem + 2 * A_ELEMS + B_ELEMS;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm = wid / Cfg::WARPS_N, wn = wid % Cfg::WARPS_N;
  la.template load<FAST>(k_begin);
  lb.template load<FAST>(k_begin);
  la.store(As0);
  lb.store(Bs0);
  __syncthreads();
  for (int t = 0; t < nk; ++t) {
    const bool odd = t & 1;
    if (t + 1 < nk) {
      la.template load<FAST>(k_begin + (t + 1) * KB);
      lb.template load<FAST>(k_begin + (t + 1) * KB);
    }
    tile_compute<T, Cfg, AMODE, BMODE>(odd ? As1 : As0, odd ? Bs1 : Bs0, wm, wn, lane, acc);
    if (t + 1 < nk) {
      la.store(odd ? As0 : As1);
      lb.store(odd ? Bs0 : Bs1);
    }
    __syncthreads();
  }
}

// Interior-tile k-loop with a DEPTH-deep register prefetch ring: tile t+DEPTH is in flight
// while tile t is multiplied, so DEPTH global-load latencies overlap instead of one (the
// one-ahead loop above is latency-bound whenever a CU holds a single workgroup and a
// k-tile is only a few MFMAs per wave - the skinny dense layers).  Plain VGPR loads: the
// compiler's counted vmcnt waits retire exactly the set being written to LDS, and the
// barrier does not drain the others.
template <int DEPTH, typename T, typename Cfg, int AMODE, int BMODE, typename LA, typename LB>
__device__ __forceinline__ void gemm_kloop_deep(LA& la, LB& lb, int k_begin, int nk, T* smem,
                                                f32x4_t (&acc)[Cfg::TM][Cfg::TN]) {
  constexpr int KB = Cfg::BK;
  constexpr int A_ELEMS = LA::Lay::ELEMS, B_ELEMS = LB::Lay::ELEMS;
  T* As[2] = {smem, smem + A_ELEMS};
  T* Bs[2] = {smem + 2 * A_ELEMS, smem + 2 * A_ELEMS + B_ELEMS};
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm = wid / Cfg::WARPS_N, wn = wid % Cfg::WARPS_N;
  u32x4_t ra[DEPTH][LA::C::NC], rb[DEPTH][LB::C::NC];
  // prologue: tile 0 -> LDS, tiles 1..DEPTH in flight (ring slot of tile j = (j - 1) % DEPTH)
  la.load_into(k_begin, ra[0]);
  lb.load_into(k_begin, rb[0]);
  la.store_from(As[0], ra[0]);
  lb.store_from(Bs[0], rb[0]);
#pragma unroll
  for (int d = 0; d < DEPTH; ++d)
    if (1 + d < nk) {
      la.load_into(k_begin + (1 + d) * KB, ra[d]);
      lb.load_into(k_begin + (1 + d) * KB, rb[d]);
    }
  __syncthreads();
  for (int t0 = 0; t0 < nk; t0 += DEPTH) {
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
      const int t = t0 + d;  // tile t + 1 sits in slot d
      if (t < nk) {
        tile_compute<T, Cfg, AMODE, BMODE>(As[t & 1], Bs[t & 1], wm, wn, lane, acc);
        if (t + 1 < nk) {
          la.store_from(As[(t + 1) & 1], ra[d]);
          lb.store_from(Bs[(t + 1) & 1], rb[d]);
          if (t + 1 + DEPTH < nk) {
            la.load_into(k_begin + (t + 1 + DEPTH) * KB, ra[d]);
            lb.load_into(k_begin + (t + 1 + DEPTH) * KB, rb[d]);
          }
        }
        __syncthreads();
      }
    }
  }
}

template <typename T, typename Cfg> struct PrefetchDepth {
  // register ring depth: ~96 VGPRs of staged tiles at most
  static constexpr int SLOT_REGS = 4 * ((Cfg::BM + Cfg::BN) * Cfg::BK * (int)sizeof(T) / 16 / GEMM_THREADS);
  static constexpr int VALUE = SLOT_REGS <= 16 ? 4 : (SLOT_REGS <= 24 ? 4 : (SLOT_REGS <= 32 ? 3 : 1));
};

template <typename T, typename Cfg, int AMODE, int BMODE, typename LA, typename LB>
__device__ __forceinline__ void gemm_mainloop(LA& la, LB& lb, int k_begin, int k_end, T* smem,
                                              f32x4_t (&acc)[Cfg::TM][Cfg::TN]) {
#pragma unroll
  for (int i = 0; i < Cfg::TM; ++i)
#pragma unroll
    for (int j = 0; j < Cfg::TN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  constexpr int KB = Cfg::BK;
  const int nk = (k_end - k_begin + KB - 1) / KB;
  if (nk <= 0) return;
  if constexpr (requires_fast_check<LA>::value && requires_fast_check<LB>::value) {
    if (la.all_fast(k_begin, k_end) && lb.all_fast(k_begin, k_end)) {
      constexpr int D = PrefetchDepth<T, Cfg>::VALUE;
      if constexpr (D > 1) {
        if (nk > 2) {
          gemm_kloop_deep<D, T, Cfg, AMODE, BMODE>(la, lb, k_begin, nk, smem, acc);
          return;
        }
      }
      gemm_kloop<true, T, Cfg, AMODE, BMODE>(la, lb, k_begin, nk, smem, acc);
      return;
    }
  }
  gemm_kloop<false, T, Cfg, AMODE, BMODE>(la, lb, k_begin, nk, smem, acc);
}

// Visit every accumulator quad: f(row0, col, f32x4 v) where row0 is the first of
// the 4 consecutive global rows and col the global column.
template <typename Cfg, typename F>
__device__ __forceinline__ void for_each_quad(int m_base, int n_base, f32x4_t (&acc)[Cfg::TM][Cfg::TN], F&& f) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm = wid / Cfg::WARPS_N, wn = wid % Cfg::WARPS_N;
#pragma unroll
  for (int i = 0; i < Cfg::TM; ++i)
#pragma unroll
    for (int j = 0; j < Cfg::TN; ++j) {
      const int row0 = m_base + wm * Cfg::WM + i * 16 + (lane >> 4) * 4;
      const int col = n_base + wn * Cfg::WN + j * 16 + (lane & 15);
      f(row0, col, acc[i][j]);
    }
}

// Map a flat block id to (tile_m, tile_n) with XCD-aware grouping so blocks
// sharing an A panel (same tile_m) run on one XCD's L2.
__device__ __forceinline__ void tile_coords(int bid, int tiles_m, int tiles_n, int& tm, int& tn) {
  const int nwg = tiles_m * tiles_n;
  const int id = xcd_remap(bid, nwg);
  tm = id / tiles_n;
  tn = id % tiles_n;
}
__device__ __forceinline__ void tile_coords(int tiles_m, int tiles_n, int& tm, int& tn) {
  tile_coords(blockIdx.x, tiles_m, tiles_n, tm, tn);
}
// The same with the tiles grouped GM m-tiles high, m fastest inside a group: the consecutive ids one
// XCD gets (xcd_remap) form a GM x (its share / GM) block, so its L2 serves every A panel and every
// B panel of the block to several workgroups (the row-major order above gives each XCD ~2 A panels
// and up to all of the B panels)
template <int GM>
__device__ __forceinline__ void tile_coords_grouped(int bid, int tiles_m, int tiles_n, int& tm, int& tn) {
  const int id = xcd_remap(bid, tiles_m * tiles_n);
  const int gsz = GM * tiles_n, grp = id / gsz, first = grp * GM;
  const int gm = tiles_m - first < GM ? tiles_m - first : GM;
  const int r = id - grp * gsz;
  tm = first + r % gm;
  tn = r / gm;
}

}  // namespace dtfe
