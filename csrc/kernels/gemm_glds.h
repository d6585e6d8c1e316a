// Dense bf16 GEMM with direct global->LDS staging (tiles 5..8 of launch_gemm_dense).
//
// Same contract and fused epilogue as gemm_dense_kernel (dense_epilogue), different main loop:
// both operands of a 64-deep k-tile are moved HBM -> LDS by global_load_lds_dwordx4 (16 B per
// lane, no VGPR staging, no ds_write pass), STAGES k-tiles in flight with a counted
// `s_waitcnt vmcnt` and a raw s_barrier per k-tile (the CDNA4 guide's glds pipeline, §5
// "Pipelining across barriers").  4 waves, 2 x 2 wave grid, 16x16x32 bf16 MFMA.
//
// LDS images are lane-linear (the DMA writes base + 16 * lane); the bank swizzle is applied
// on the SOURCE address and undone on the fragment read (rule 21):
//   KMAJ operand (k contiguous): [R rows][64 k] 128-B rows, slot s of row r holds logical
//        16-B chunk s ^ (r & 7) -> ds_read_b128 fragment reads hit 16 distinct slots
//   RMAJ operand (rows contiguous): [64 k][R] read with ds_read_b64_tr_b16, the 16-B chunks
//        of k-row k XOR-ed by an even h(k) so a 32-lane half covers 8 distinct 32-B segments
// A whole n-tile (or m-tile) may be a "ones tile": the bias column of a weight-gradient GEMM
// (b_ones_row) lies past the operand's last row, so every load of that tile reads a page of
// bf16 ones (the other columns of the tile are discarded by the epilogue).
//
// Used by the MNIST-CNN fc1 forward / data-gradient / weight-gradient GEMMs
// (M, N in {1024, 3136}, K in {1024, 3136}) - the reference network's dense layers
// (SURVEY K01-K03).
#pragma once
#include "gemm_dense.h"

namespace dtfe {

constexpr int GL_BK = 64;
typedef __attribute__((address_space(3))) void gl_lds_t;

__device__ __forceinline__ void gl_dma16(const void* g, bf16* lds_piece) {
  __builtin_amdgcn_global_load_lds(g, (gl_lds_t*)lds_piece, 16, 0, 0);
}

// chunk XOR of k-row k in a [64 k][COLS] RMAJ image
template <int COLS> __device__ __forceinline__ int gl_rswz(int k) {
  if constexpr (COLS == 128) return 2 * ((k & 3) | (((k >> 3) & 1) << 2));
  else return 2 * (((k >> 1) & 1) | (((k >> 3) & 1) << 1));
}

// One operand of the glds GEMM: R rows of the block tile, MODE = global layout.
template <int R, int MODE>
struct GlOperand {
  static constexpr int NP = R / 32;         // 1-KB DMA pieces per thread and k-tile
  static constexpr int ELEMS = R * GL_BK;   // image elements per stage
  const bf16* src[NP];                      // this lane's source at k0 = 0 (or the ones page)
  long kstep;                               // source advance per k-tile (elements)

  __device__ __forceinline__ void init(const bf16* p, long ld, int r0, int w, int lane, const bf16* ones,
                                       bool ones_tile) {
    if constexpr (MODE == KMAJ) {
      const int lrow = lane >> 3, lchunk = (lane & 7) ^ lrow;
#pragma unroll
      for (int j = 0; j < NP; ++j) {
        const int row = (j * 4 + w) * 8 + lrow;
        src[j] = ones_tile ? ones + lchunk * 8 : p + (long)(r0 + row) * ld + lchunk * 8;
      }
      kstep = ones_tile ? 0 : GL_BK;
    } else {
      constexpr int CPR = R / 8, RPP = 64 / CPR;
#pragma unroll
      for (int j = 0; j < NP; ++j) {
        const int krow = (j * 4 + w) * RPP + lane / CPR;
        const int chunk = (lane % CPR) ^ gl_rswz<R>(krow);
        src[j] = ones_tile ? ones + chunk * 8 : p + (long)krow * ld + r0 + chunk * 8;
      }
      kstep = ones_tile ? 0 : GL_BK * ld;
    }
  }
  __device__ __forceinline__ void issue(int kt, bf16* img, int w) const {
#pragma unroll
    for (int j = 0; j < NP; ++j) gl_dma16(src[j] + kt * kstep, img + (j * 4 + w) * 512);
  }
  // 16x16x32 fragment of rows rbase.. at k-step kk (0 or 1) of the image
  __device__ __forceinline__ bf16x8_t frag(const bf16* img, int rbase, int kk, int lane) const {
    if constexpr (MODE == KMAJ) {
      const int pc = (kk * 4 + (lane >> 4)) ^ (lane & 7);
      return *reinterpret_cast<const bf16x8_t*>(img + (rbase + (lane & 15)) * GL_BK + pc * 8);
    } else {
      const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
      const int c = rbase + 4 * p;
      const int k0 = kk * 32 + 8 * g + q, k1 = k0 + 4;
      const bf16* p0 = img + k0 * R + (c ^ (gl_rswz<R>(k0) * 8));
      const bf16* p1 = img + k1 * R + (c ^ (gl_rswz<R>(k1) * 8));
      s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4_t, p0));
      s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4_t, p1));
      s16x8_t v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      return __builtin_bit_cast(bf16x8_t, v);
    }
  }
};

template <int BM, int BN, int STAGES> struct GlSmem {
  static constexpr int STAGE_EL = (BM + BN) * GL_BK;
  static constexpr int STAGING = STAGES * STAGE_EL * 2;
  static constexpr int CTILE = BM * (BN + 4) * 4;
  static constexpr int BYTES = STAGING > CTILE ? STAGING : CTILE;
};

// One output tile (workgroup `bid` of this GEMM's grid); smem_raw: GlSmem<BM, BN, STAGES>::BYTES of LDS.
// Shared by the plain launch below and the grouped launch (gemm_glds_group_kernel).
template <int BM, int BN, int AMODE, int BMODE, int STAGES>
__device__ __forceinline__ void gemm_glds_body(const DenseGemmArgs& a, int bid, char* smem_raw) {
  using Cfg = TileCfg<bf16, BM, BN, 2, 2, GL_BK>;
  using OA = GlOperand<BM, AMODE>;
  using OB = GlOperand<BN, BMODE>;
  constexpr int NPT = OA::NP + OB::NP;  // DMA instructions per thread and k-tile
  using SM = GlSmem<BM, BN, STAGES>;
  bf16* smem = reinterpret_cast<bf16*>(smem_raw);

  const int tiles_m = a.M / BM, tiles_n = (a.N + BN - 1) / BN;
  int tm, tn;
  tile_coords(bid, tiles_m, tiles_n, tm, tn);
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int m_base = tm * BM, n_base = tn * BN;
  const int kt0 = blockIdx.z * (a.k_chunk / GL_BK);
  const int nk = min(a.K, (int)(blockIdx.z + 1) * a.k_chunk) / GL_BK - kt0;

  OA oa;
  OB ob;
  oa.init((const bf16*)a.A + (AMODE == KMAJ ? (long)kt0 * GL_BK : (long)kt0 * GL_BK * a.lda), a.lda, m_base, w,
          lane, a.ones, false);
  ob.init((const bf16*)a.B + (BMODE == KMAJ ? (long)kt0 * GL_BK : (long)kt0 * GL_BK * a.ldb), a.ldb, n_base, w,
          lane, a.ones, a.b_ones_row >= 0 && n_base == a.b_ones_row);

  f32x4_t acc[Cfg::TM][Cfg::TN];
#pragma unroll
  for (int i = 0; i < Cfg::TM; ++i)
#pragma unroll
    for (int j = 0; j < Cfg::TN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  auto stage_a = [&](int s) { return smem + s * SM::STAGE_EL; };
  auto stage_b = [&](int s) { return smem + s * SM::STAGE_EL + OA::ELEMS; };
#pragma unroll
  for (int s = 0; s < STAGES - 1; ++s)
    if (s < nk) {
      oa.issue(s, stage_a(s), w);
      ob.issue(s, stage_b(s), w);
    }
  const int wm = w >> 1, wn = w & 1;
  int cur = 0;
  for (int t = 0; t < nk; ++t) {
    // tile t landed (this wave's pieces: counted wait leaving the younger tiles in flight),
    // then a barrier so every wave's pieces of tile t are visible and tile t-1's buffer is free
    if (t + STAGES - 2 < nk) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"((STAGES - 2) * NPT) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (t + STAGES - 1 < nk) {
      int s = cur + STAGES - 1;
      if (s >= STAGES) s -= STAGES;
      oa.issue(t + STAGES - 1, stage_a(s), w);
      ob.issue(t + STAGES - 1, stage_b(s), w);
    }
    const bf16* As = stage_a(cur);
    const bf16* Bs = stage_b(cur);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8_t af[Cfg::TM], bfr[Cfg::TN];
#pragma unroll
      for (int i = 0; i < Cfg::TM; ++i) af[i] = oa.frag(As, wm * Cfg::WM + i * 16, kk, lane);
#pragma unroll
      for (int j = 0; j < Cfg::TN; ++j) bfr[j] = ob.frag(Bs, wn * Cfg::WN + j * 16, kk, lane);
#pragma unroll
      for (int i = 0; i < Cfg::TM; ++i)
#pragma unroll
        for (int j = 0; j < Cfg::TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    cur = cur + 1 == STAGES ? 0 : cur + 1;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();  // the epilogue reuses the staging LDS for the C tile
  dense_epilogue<Cfg>(a, smem_raw, acc, tm, tn, tiles_m, tiles_n);
}

template <int BM, int BN, int AMODE, int BMODE, int STAGES>
__global__ __launch_bounds__(GEMM_THREADS, 1) void gemm_glds_kernel(DenseGemmArgs a) {
  __shared__ __attribute__((aligned(16))) char smem_raw[GlSmem<BM, BN, STAGES>::BYTES];
  gemm_glds_body<BM, BN, AMODE, BMODE, STAGES>(a, blockIdx.x, smem_raw);
}

}  // namespace dtfe
