// Tile 22: the 8-wave 256x128 global_load_lds GEMM of the MNIST-CNN fc1 layer (see gemm_fc.h), and
// the grouped fc backward launch built on it (head weight gradient + fc1 data / weight gradients).
#include "gemm_fc.h"

#include <cstring>
#include <stdexcept>

namespace dtfe {

namespace fcg {

constexpr int KT = 64;      // k-tile depth (2 MFMA k-steps)
constexpr int STAGES = 3;   // k-tiles in flight per workgroup
constexpr int NWAVE = 8;

// the 4 x 2 wave grid of the 256 x 128 tile (64 x 64 per wave, 4 x 4 accumulators of 16 x 16);
// member names follow TileCfg so dense_epilogue can take it
struct FcCfg {
  static constexpr int BM = FC_BM, BN = FC_BN, WARPS_M = 4, WARPS_N = 2;
  static constexpr int WM = BM / WARPS_M, WN = BN / WARPS_N, TM = WM / 16, TN = WN / 16;
  static constexpr int WAVES = NWAVE;
};

constexpr int STAGE_EL = (FC_BM + FC_BN) * KT;                 // bf16 elements of one stage
constexpr int STAGING_BYTES = STAGES * STAGE_EL * 2;            // 144 KB
constexpr int CTILE_BYTES = FC_BM * (FC_BN + 4) * 4;            // 132 KB (epilogue's f32 C tile)
constexpr int SMEM_BYTES = STAGING_BYTES > CTILE_BYTES ? STAGING_BYTES : CTILE_BYTES;

// chunk XOR of k-row k in a [64 k][COLS >= 128] RMAJ image: the 8 k-rows one 32-lane half of a
// ds_read_b64_tr_b16 touches land on 8 distinct 32-B bank groups (rows are multiples of 256 B)
__device__ __forceinline__ int rswz(int k) { return 2 * ((k & 3) | (((k >> 3) & 1) << 2)); }

// One operand of the tile: R rows, global layout MODE.  A k-tile is R / 8 pieces of 1 KB (one
// global_load_lds_dwordx4 wave-instruction each, lane-linear in LDS), R / 64 per wave.
//   KMAJ (k contiguous): piece = 8 rows x 64 k, slot s of row r holds logical 16-B chunk s ^ (r & 7)
//   RMAJ (rows contiguous): piece = 64 / (R / 8) k-rows x R columns, chunk c of k-row k at c ^ rswz(k)
// RMAJ sources past the valid columns are clamped into the row (their outputs are never stored);
// the chunk that starts at `ones_col` reads the ones page instead (bias column of a weight gradient).
template <int R, int MODE>
struct FcOperand {
  static constexpr int NP = R / 64;
  static constexpr int ELEMS = R * KT;
  const bf16* src[NP];
  long kstep[NP];

  __device__ __forceinline__ void init(const bf16* p, long ld, int r0, int valid, int ones_col, const bf16* ones,
                                       int w, int lane) {
#pragma unroll
    for (int j = 0; j < NP; ++j) {
      const int piece = j * NWAVE + w;
      if constexpr (MODE == KMAJ) {
        const int lrow = lane >> 3, lchunk = (lane & 7) ^ lrow;
        src[j] = p + (long)(r0 + piece * 8 + lrow) * ld + lchunk * 8;
        kstep[j] = KT;
      } else {
        constexpr int CPR = R / 8, RPP = 64 / CPR;
        const int krow = piece * RPP + lane / CPR;
        const int chunk = (lane % CPR) ^ rswz(krow);
        int col = r0 + chunk * 8;
        if (col == ones_col) {
          src[j] = ones;
          kstep[j] = 0;
          continue;
        }
        if (col + 8 > valid) col = valid - 8;
        src[j] = p + (long)krow * ld + col;
        kstep[j] = (long)KT * ld;
      }
    }
  }
  // the DMA from inline asm (M0 = the wave-uniform LDS destination), as igemm.hip's glds16_async:
  // with the builtin, the compiler's LDS-DMA alias tracking puts an `s_waitcnt vmcnt(0)` in front of
  // every ds_read_b64_tr_b16 (that builtin carries no memory operand), draining the whole prefetch
  // ring each k-tile; fc_body orders every stage with its own counted vmcnt wait + barrier
  __device__ __forceinline__ void issue(int kt, bf16* img, int w) const {
#pragma unroll
    for (int j = 0; j < NP; ++j) {
      const uint32_t l = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(img + (j * NWAVE + w) * 512));
      asm volatile("global_load_lds_dwordx4 %0, off" ::"v"(src[j] + kt * kstep[j]), "{m0}"(l) : "memory");
    }
  }
  // 16x16x32 fragment of rows rbase.. at k-step kk (0 or 1)
  __device__ __forceinline__ bf16x8_t frag(const bf16* img, int rbase, int kk, int lane) const {
    if constexpr (MODE == KMAJ) {
      const int pc = (kk * 4 + (lane >> 4)) ^ (lane & 7);
      return *reinterpret_cast<const bf16x8_t*>(img + (rbase + (lane & 15)) * KT + pc * 8);
    } else {
      const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
      const int c = rbase + 4 * p;
      const int k0 = kk * 32 + 8 * g + q, k1 = k0 + 4;
      const bf16* p0 = img + k0 * R + (c ^ (rswz(k0) * 8));
      const bf16* p1 = img + k1 * R + (c ^ (rswz(k1) * 8));
      s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4_t, p0));
      s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4_t, p1));
      s16x8_t v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      return __builtin_bit_cast(bf16x8_t, v);
    }
  }
};

// One 256 x 128 output tile (workgroup `bid` of this GEMM, split blockIdx.z): the glds pipeline of
// gemm_glds_body (counted vmcnt + one raw s_barrier per k-tile, STAGES - 1 k-tiles in flight)
// with 8 waves, then the shared dense epilogue (bias / activation / dropout / act' / split-K / bias
// column routing).
template <int AMODE, int BMODE>
__device__ __forceinline__ void fc_body(const DenseGemmArgs& a, int bid, char* smem_raw) {
  using OA = FcOperand<FC_BM, AMODE>;
  using OB = FcOperand<FC_BN, BMODE>;
  constexpr int NPT = OA::NP + OB::NP;  // DMA instructions per thread and k-tile
  bf16* smem = reinterpret_cast<bf16*>(smem_raw);
  const int tiles_m = a.M / FC_BM, tiles_n = (a.N + FC_BN - 1) / FC_BN;
  // XCD-aware order, m fastest: the ~12 consecutive tiles one XCD gets (xcd_remap) are every m-tile
  // of 3-4 n-tiles, so its L2 serves each B panel to all m-tiles (the default n-fastest order gave
  // each XCD 12 private B panels: TCC hit rate 55 %, profiles/r6_fc1_tile22.txt)
  const int id = xcd_remap(bid, tiles_m * tiles_n);
  const int tm = id % tiles_m, tn = id / tiles_m;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int m_base = tm * FC_BM, n_base = tn * FC_BN;
  const int kt0 = blockIdx.z * (a.k_chunk / KT);
  const int nk = min(a.K, (int)(blockIdx.z + 1) * a.k_chunk) / KT - kt0;
  // the B operand's real columns: the bias column (b_ones_row = N - 1) is not a row of B
  const int b_valid = a.b_ones_row >= 0 ? a.b_ones_row : a.N;

  OA oa;
  OB ob;
  oa.init((const bf16*)a.A + (AMODE == KMAJ ? (long)kt0 * KT : (long)kt0 * KT * a.lda), a.lda, m_base, a.M, -1,
          a.ones, w, lane);
  ob.init((const bf16*)a.B + (BMODE == KMAJ ? (long)kt0 * KT : (long)kt0 * KT * a.ldb), a.ldb, n_base, b_valid,
          a.b_ones_row, a.ones, w, lane);

  f32x4_t acc[FcCfg::TM][FcCfg::TN];
#pragma unroll
  for (int i = 0; i < FcCfg::TM; ++i)
#pragma unroll
    for (int j = 0; j < FcCfg::TN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // (stage s: A image at smem + s * STAGE_EL, B image right after it)
#pragma unroll
  for (int s = 0; s < STAGES - 1; ++s)
    if (s < nk) {
      oa.issue(s, smem + s * STAGE_EL, w);
      ob.issue(s, smem + s * STAGE_EL + OA::ELEMS, w);
    }
  const int wm = w >> 1, wn = w & 1;
  int cur = 0;
  for (int t = 0; t < nk; ++t) {
    // tile t landed (this wave's pieces; the younger tiles stay in flight), then a barrier so every
    // wave's pieces are visible and the slot read in iteration t - 1 is free for tile t + STAGES - 1
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
      oa.issue(t + STAGES - 1, smem + s * STAGE_EL, w);
      ob.issue(t + STAGES - 1, smem + s * STAGE_EL + OA::ELEMS, w);
    }
    const bf16* As = smem + cur * STAGE_EL;
    const bf16* Bs = As + OA::ELEMS;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8_t af[FcCfg::TM], bfr[FcCfg::TN];
#pragma unroll
      for (int i = 0; i < FcCfg::TM; ++i) af[i] = oa.frag(As, wm * FcCfg::WM + i * 16, kk, lane);
#pragma unroll
      for (int j = 0; j < FcCfg::TN; ++j) bfr[j] = ob.frag(Bs, wn * FcCfg::WN + j * 16, kk, lane);
#pragma unroll
      for (int i = 0; i < FcCfg::TM; ++i)
#pragma unroll
        for (int j = 0; j < FcCfg::TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    cur = cur + 1 == STAGES ? 0 : cur + 1;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();  // the epilogue reuses the staging LDS for the C tile
  dense_epilogue<FcCfg, FC_THREADS>(a, smem_raw, acc, tm, tn, tiles_m, tiles_n);
}

template <int AMODE, int BMODE>
__global__ __launch_bounds__(FC_THREADS, 1) void gemm_fc_kernel(DenseGemmArgs a) {
  __shared__ __attribute__((aligned(16))) char smem_raw[SMEM_BYTES];
  fc_body<AMODE, BMODE>(a, blockIdx.x, smem_raw);
}


// Head weight gradient, one WAVE per 4 columns of dW (piece p: columns 4p..4p+3; p == K / 4: the
// bias), the whole batch streamed by the wave's 64 lanes - 40 accumulators, no cross-wave reduce.
// The bias piece also folds head_xent's loss / hit partials (it must run on wave 0: head_fold_parts).
template <int NC>
__device__ __forceinline__ void head_wgrad_wave_body(const HeadWgradArgs& a, int piece) {
  static_assert(NC * 4 == 40, "the butterfly below is laid out for 10 classes x 4 columns");
  constexpr int V = NC * 4;
  const int lane = threadIdx.x & 63;
  const bool bias_blk = piece * 4 >= a.K;
  const int col0 = bias_blk ? 0 : piece * 4;
  float v[V];
#pragma unroll
  for (int j = 0; j < V; ++j) v[j] = 0.f;
#pragma unroll 4
  for (int b0 = 0; b0 < a.B; b0 += 64) {
    const int b = b0 + lane;
    const bool ok = b < a.B;
    const long r = ok ? b : 0;  // clamped row: loads stay in bounds, the products are zeroed
    const u32x2_t hv = *reinterpret_cast<const u32x2_t*>(a.h + r * a.ldh + col0);
    const u32x4_t d0 = *reinterpret_cast<const u32x4_t*>(a.dl + r * a.ld_dl);
    const uint32_t d1 = *reinterpret_cast<const uint32_t*>(a.dl + r * a.ld_dl + 8);
    float h[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) h[e] = !ok ? 0.f : bias_blk ? 1.f : bf2f((bf16)(hv[e >> 1] >> (16 * (e & 1))));
#pragma unroll
    for (int n = 0; n < NC; ++n) {
      const uint32_t wv = n < 8 ? d0[n >> 1] : d1;
      const float d = bf2f((bf16)(wv >> (16 * (n & 1))));
#pragma unroll
      for (int e = 0; e < 4; ++e) v[n * 4 + e] = fmaf(d, h[e], v[n * 4 + e]);
    }
  }
  // halving butterfly over lane bits 5..3: 40 -> 20 -> 10 -> 5 values per lane, then bits 2..0
  auto halve = [&](auto half_c, int mask) {
    constexpr int H = decltype(half_c)::value;
    const bool hi = (lane & mask) != 0;
#pragma unroll
    for (int j = 0; j < H; ++j) {
      const float send = hi ? v[j] : v[H + j];
      const float keep = hi ? v[H + j] : v[j];
      v[j] = keep + __shfl_xor(send, mask, 64);
    }
  };
  halve(std::integral_constant<int, 20>{}, 32);
  halve(std::integral_constant<int, 10>{}, 16);
  halve(std::integral_constant<int, 5>{}, 8);
#pragma unroll
  for (int j = 0; j < 5; ++j) {
    v[j] += __shfl_xor(v[j], 4, 64);
    v[j] += __shfl_xor(v[j], 2, 64);
    v[j] += __shfl_xor(v[j], 1, 64);
  }
  // lane holds values ((b5 ? 20 : 0) + (b4 ? 10 : 0) + (b3 ? 5 : 0) + j), value index = n * 4 + e
  if ((lane & 7) == 0) {
    const int base = ((lane >> 5) & 1) * 20 + ((lane >> 4) & 1) * 10 + ((lane >> 3) & 1) * 5;
#pragma unroll
    for (int j = 0; j < 5; ++j) {
      const int idx = base + j, n = idx >> 2, e = idx & 3;
      if (!bias_blk) a.dw[(long)n * a.ldw + col0 + e] = v[j] * a.scale;
      else if (e == 0) a.db[n] = v[j] * a.scale;
    }
  }
  if (bias_blk) head_fold_parts(a);
}

// The grouped fc backward: workgroups [0, nh) the head weight gradient (8 pieces each), then the
// (KMAJ, RMAJ) GEMM's tiles (fc1 data gradient), then the (RMAJ, RMAJ) GEMM's (fc1 weight gradient).
// Every piece fits the machine at once (33 + 100 + 100 workgroups at B = 1024), one per CU.
struct FcGroupArgs {
  DenseGemmArgs g0, g1;
  HeadWgradArgs h;
  int nh, n0, n1;     // padded workgroup ranges
  int ph, t0, t1;     // head pieces (waves), real GEMM tiles
};

template <bool HEAD>
__global__ __launch_bounds__(FC_THREADS, 1) void gemm_fc_group_kernel(FcGroupArgs ga) {
  __shared__ __attribute__((aligned(16))) char smem_raw[SMEM_BYTES];
  int bid = blockIdx.x;
  if constexpr (HEAD) {
    if (bid < ga.nh) {
      const int piece = bid * NWAVE + (int)(threadIdx.x >> 6);
      if (piece < ga.ph) head_wgrad_wave_body<10>(ga.h, piece);
      return;
    }
    bid -= ga.nh;
  }
  if (bid < ga.n0) {
    if (bid < ga.t0) fc_body<KMAJ, RMAJ>(ga.g0, bid, smem_raw);
    return;
  }
  bid -= ga.n0;
  if (bid < ga.t1) fc_body<RMAJ, RMAJ>(ga.g1, bid, smem_raw);
}

int tiles_of(const DenseGemmArgs& a) { return (a.M / FC_BM) * ((a.N + FC_BN - 1) / FC_BN); }
int pad8(int n) { return (n + 7) / 8 * 8; }

}  // namespace fcg

using namespace fcg;

bool gemm_fc_eligible(int dtype, int amode, int bmode, const DenseGemmArgs& a) {
  if (dtype != 0 || a.a_ones_row >= 0 || a.M % FC_BM || a.K % KT || a.k_chunk % KT) return false;
  if ((a.lda % 8) || (a.ldb % 8) || (((uintptr_t)a.A) & 15) || (((uintptr_t)a.B) & 15)) return false;
  const int b_valid = a.b_ones_row >= 0 ? a.b_ones_row : a.N;
  if (a.b_ones_row >= 0 && (a.b_ones_row != a.N - 1 || a.b_ones_row % 8 || !a.ones || (((uintptr_t)a.ones) & 15)))
    return false;
  if (b_valid < 8 || b_valid % 8) return false;
  if (bmode == KMAJ && (a.N % FC_BN || a.b_ones_row >= 0)) return false;  // KMAJ B: whole n-tiles only
  if (amode != KMAJ && amode != RMAJ) return false;
  return true;
}

void launch_gemm_fc(int amode, int bmode, int splits, const DenseGemmArgs& a, hipStream_t s) {
  if (splits < 1) splits = 1;
  if (splits > 1 && !a.atomic && (!a.ws || !a.tile_ctr))
    throw std::runtime_error("gemm_fc: split-K with a fused epilogue needs a workspace");
  dim3 grid(tiles_of(a), 1, splits);
  if (amode == KMAJ && bmode == KMAJ) hipLaunchKernelGGL((gemm_fc_kernel<KMAJ, KMAJ>), grid, dim3(FC_THREADS), 0, s, a);
  else if (amode == KMAJ && bmode == RMAJ) hipLaunchKernelGGL((gemm_fc_kernel<KMAJ, RMAJ>), grid, dim3(FC_THREADS), 0, s, a);
  else if (amode == RMAJ && bmode == KMAJ) hipLaunchKernelGGL((gemm_fc_kernel<RMAJ, KMAJ>), grid, dim3(FC_THREADS), 0, s, a);
  else hipLaunchKernelGGL((gemm_fc_kernel<RMAJ, RMAJ>), grid, dim3(FC_THREADS), 0, s, a);
}

void launch_gemm_fc_group(const DenseGemmArgs& g0, const DenseGemmArgs& g1, const HeadWgradArgs* h, hipStream_t s) {
  FcGroupArgs ga;
  std::memset(&ga, 0, sizeof(ga));
  ga.g0 = g0;
  ga.g1 = g1;
  ga.t0 = tiles_of(g0);
  ga.t1 = tiles_of(g1);
  ga.n0 = pad8(ga.t0);
  ga.n1 = ga.t1;
  if (h) {
    ga.h = *h;
    ga.ph = h->K / 4 + (h->db ? 1 : 0);
    ga.nh = pad8((ga.ph + NWAVE - 1) / NWAVE);
    hipLaunchKernelGGL((gemm_fc_group_kernel<true>), dim3(ga.nh + ga.n0 + ga.n1), dim3(FC_THREADS), 0, s, ga);
  } else {
    hipLaunchKernelGGL((gemm_fc_group_kernel<false>), dim3(ga.n0 + ga.n1), dim3(FC_THREADS), 0, s, ga);
  }
}

}  // namespace dtfe
