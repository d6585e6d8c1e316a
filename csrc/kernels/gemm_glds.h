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

// The DMA is issued from inline asm (M0 = the wave-uniform LDS destination), as igemm.hip's
// glds16_async: with the builtin, the compiler's LDS-DMA alias tracking puts an `s_waitcnt vmcnt(0)`
// in front of every ds_read_b64_tr_b16 of an RMAJ operand (that builtin carries no memory operand),
// draining the whole prefetch ring each k-tile.  gemm_glds_body orders every stage with its own
// counted vmcnt wait + barrier; the compiler's own vmcnt waits stay conservative (these are older).
__device__ __forceinline__ void gl_dma16(const void* g, bf16* lds_piece) {
  const uint32_t l = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)lds_piece);
  asm volatile("global_load_lds_dwordx4 %0, off" ::"v"(g), "{m0}"(l) : "memory");
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

template <int BM, int BN, int STAGES, int KG = 1> struct GlSmem {
  static constexpr int STAGE_EL = (BM + BN) * GL_BK;
  static constexpr int STAGING = KG * STAGES * STAGE_EL * 2;
  static constexpr int CTILE = BM * (BN + 4) * 4;
  static constexpr int BYTES = STAGING > CTILE ? STAGING : CTILE;
};

// One output tile (workgroup `bid` of this GEMM's grid); smem_raw: GlSmem<BM, BN, STAGES, KG>::BYTES of LDS.
// Shared by the plain launch below and the grouped launch (gemm_glds_group_kernel).
//
// KG > 1: KG groups of 4 waves (256 * KG threads) split the workgroup's k-tiles round-robin, each
// group with its own STAGES-deep ring, and fold their accumulators through LDS before the
// epilogue.  The global -> LDS DMA rate of a CU grows with the number of waves issuing it, not
// with the ring depth of one wave (profiles/r3_cnn_kernel_tuning.txt: 1 workgroup per CU streams
// 20-30 B/clk whatever its depth, 3 workgroups 35-44): a long-K GEMM with ~one tile per CU (the
// MNIST fc1 forward) gets the extra waves without splitting K across workgroups.
template <int BM, int BN, int AMODE, int BMODE, int STAGES, int KG = 1>
__device__ __forceinline__ void gemm_glds_body(const DenseGemmArgs& a, int bid, char* smem_raw) {
  using Cfg = TileCfg<bf16, BM, BN, 2, 2, GL_BK>;
  using OA = GlOperand<BM, AMODE>;
  using OB = GlOperand<BN, BMODE>;
  constexpr int NPT = OA::NP + OB::NP;  // DMA instructions per thread and k-tile
  using SM = GlSmem<BM, BN, STAGES, KG>;
  bf16* smem = reinterpret_cast<bf16*>(smem_raw);
  const int kg = KG > 1 ? __builtin_amdgcn_readfirstlane(threadIdx.x >> 8) : 0;  // k-group of this wave

  const int tiles_m = a.M / BM, tiles_n = (a.N + BN - 1) / BN;
  int tm, tn;
  tile_coords_grouped<4>(bid, tiles_m, tiles_n, tm, tn);
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane((threadIdx.x >> 6) & 3);
  const int m_base = tm * BM, n_base = tn * BN;
  const int kt0 = blockIdx.z * (a.k_chunk / GL_BK);
  const int nk_all = min(a.K, (int)(blockIdx.z + 1) * a.k_chunk) / GL_BK - kt0;
  // this group's k-tiles: kg, kg + KG, ... (local index t -> k-tile kg + t * KG); the loop runs the
  // largest group's count so every wave meets every barrier
  const int nk = (nk_all - kg + KG - 1) / KG;
  const int nloop = (nk_all + KG - 1) / KG;

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

  bf16* ring = smem + kg * STAGES * SM::STAGE_EL;
  auto stage_a = [&](int s) { return ring + s * SM::STAGE_EL; };
  auto stage_b = [&](int s) { return ring + s * SM::STAGE_EL + OA::ELEMS; };
#pragma unroll
  for (int s = 0; s < STAGES - 1; ++s)
    if (s < nk) {
      oa.issue(kg + s * KG, stage_a(s), w);
      ob.issue(kg + s * KG, stage_b(s), w);
    }
  const int wm = w >> 1, wn = w & 1;
  int cur = 0;
  for (int t = 0; t < nloop; ++t) {
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
      oa.issue(kg + (t + STAGES - 1) * KG, stage_a(s), w);
      ob.issue(kg + (t + STAGES - 1) * KG, stage_b(s), w);
    }
    if (KG > 1 && t >= nk) continue;  // (a group one k-tile short: still at every barrier)
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
  if constexpr (KG > 1) {
    // groups 1.. park their accumulators lane-linearly in LDS, group 0 adds them in group order
    constexpr int FR = Cfg::TM * Cfg::TN;
    f32x4_t* park = reinterpret_cast<f32x4_t*>(smem_raw);
    if (kg > 0) {
#pragma unroll
      for (int i = 0; i < Cfg::TM; ++i)
#pragma unroll
        for (int j = 0; j < Cfg::TN; ++j) park[(((kg - 1) * 4 + w) * FR + i * Cfg::TN + j) * 64 + lane] = acc[i][j];
    }
    __syncthreads();
    if (kg == 0) {
      for (int g = 1; g < KG; ++g)
#pragma unroll
        for (int i = 0; i < Cfg::TM; ++i)
#pragma unroll
          for (int j = 0; j < Cfg::TN; ++j) acc[i][j] += park[(((g - 1) * 4 + w) * FR + i * Cfg::TN + j) * 64 + lane];
    }
    __syncthreads();
  }
  dense_epilogue<Cfg, GEMM_THREADS * KG>(a, smem_raw, acc, tm, tn, tiles_m, tiles_n);
}

template <int BM, int BN, int AMODE, int BMODE, int STAGES, int KG = 1>
__global__ __launch_bounds__(GEMM_THREADS * KG, 1) void gemm_glds_kernel(DenseGemmArgs a) {
  __shared__ __attribute__((aligned(16))) char smem_raw[GlSmem<BM, BN, STAGES, KG>::BYTES];
  gemm_glds_body<BM, BN, AMODE, BMODE, STAGES, KG>(a, blockIdx.x, smem_raw);
}

}  // namespace dtfe
