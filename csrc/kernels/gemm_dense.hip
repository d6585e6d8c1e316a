// Instantiation + dispatch of the dense GEMM kernel family.
#include "gemm_dense.h"
#include "gemm_glds.h"
#include "gemm_fc.h"
#include "head.h"

#include <cstring>
#include <stdexcept>

namespace dtfe {

template <typename T, typename Cfg, int AM, int BMD>
static void launch_one(int splits, const DenseGemmArgs& args, hipStream_t s) {
  const int tiles = ((args.M + Cfg::BM - 1) / Cfg::BM) * ((args.N + Cfg::BN - 1) / Cfg::BN);
  if (args.k_chunk % Cfg::BK) throw std::runtime_error("gemm_dense: split-K chunk must be a multiple of the k-tile");
  if (splits > 1 && !args.atomic && (!args.ws || !args.tile_ctr))
    throw std::runtime_error("gemm_dense: split-K with a fused epilogue needs a workspace");
  dim3 grid(tiles, 1, splits);
  hipLaunchKernelGGL((gemm_dense_kernel<T, Cfg, AM, BMD>), grid, dim3(GEMM_THREADS), 0, s, args);
}

int gemm_dense_tile_dims(int tile, int& bm, int& bn) {
  static const int dims[23][2] = {{64, 64}, {128, 128}, {128, 64}, {64, 128}, {32, 32},
                                  {128, 128}, {128, 64}, {64, 128}, {64, 64},
                                  {128, 128}, {128, 64}, {64, 128}, {64, 64}, {16, 16},
                                  {64, 64}, {64, 64}, {64, 64}, {128, 64}, {128, 64},
                                  {64, 64}, {64, 64}, {64, 64}, {FC_BM, FC_BN}};
  if (tile < 0 || tile > FC_TILE) return -1;
  bm = dims[tile][0];
  bn = dims[tile][1];
  if (tile == GEMM_TILE_SMALL) return 16;
  return tile >= 5 ? GL_BK : GEMM_KTILE;
}

bool gemm_glds_eligible(int dtype, int amode, int bmode, int tile, const DenseGemmArgs& a) {
  if (tile == FC_TILE) return gemm_fc_eligible(dtype, amode, bmode, a);
  int bm = 0, bn = 0;
  if (tile < 5 || gemm_dense_tile_dims(tile, bm, bn) < 0) return false;
  if (dtype != 0 || a.a_ones_row >= 0 || a.K % GL_BK || a.k_chunk % GL_BK || a.M % bm) return false;
  if ((a.lda % 8) || (a.ldb % 8) || (((uintptr_t)a.A) & 15) || (((uintptr_t)a.B) & 15)) return false;
  // n-tiles: whole tiles of real rows, plus at most one trailing tile that starts at the ones row
  if (a.b_ones_row >= 0) {
    if (a.b_ones_row != a.N - 1 || a.b_ones_row % bn || !a.ones || (((uintptr_t)a.ones) & 15)) return false;
  } else if (a.N % bn) {
    return false;
  }
  (void)amode;
  (void)bmode;
  return true;
}

// tiles 5..8: 3 k-tiles in flight (one workgroup per CU streams deeper);
// tiles 9..12: 2 stages, half the LDS, so more workgroups share a CU (grids of many tiles);
// tiles 14..18: deeper pipelines (64x64 with 4 / 6 / 8 stages, 128x64 with 4 / 6) for long-K grids
// of about one workgroup per CU, where 3 stages leave the k-loop waiting on the load latency
// tiles 19..21: 64x64 with 2 / 4 k-groups of 4 waves splitting the k-tiles inside the workgroup
// (3 / 2 / 4 stages per group): more waves issuing global->LDS DMA per CU for ~one tile per CU
template <int BM, int BN, int AM, int BMD, int STAGES, int KG = 1>
static void launch_glds(int splits, const DenseGemmArgs& a, hipStream_t s) {
  const int tiles = (a.M / BM) * ((a.N + BN - 1) / BN);
  dim3 grid(tiles, 1, splits);
  hipLaunchKernelGGL((gemm_glds_kernel<BM, BN, AM, BMD, STAGES, KG>), grid, dim3(GEMM_THREADS * KG), 0, s, a);
}

template <int AM, int BMD>
static void glds_by_tile(int tile, int splits, const DenseGemmArgs& a, hipStream_t s) {
  switch (tile) {
    case 5: launch_glds<128, 128, AM, BMD, 3>(splits, a, s); break;
    case 6: launch_glds<128, 64, AM, BMD, 3>(splits, a, s); break;
    case 7: launch_glds<64, 128, AM, BMD, 3>(splits, a, s); break;
    case 8: launch_glds<64, 64, AM, BMD, 3>(splits, a, s); break;
    case 9: launch_glds<128, 128, AM, BMD, 2>(splits, a, s); break;
    case 10: launch_glds<128, 64, AM, BMD, 2>(splits, a, s); break;
    case 11: launch_glds<64, 128, AM, BMD, 2>(splits, a, s); break;
    case 12: launch_glds<64, 64, AM, BMD, 2>(splits, a, s); break;
    case 14: launch_glds<64, 64, AM, BMD, 4>(splits, a, s); break;
    case 15: launch_glds<64, 64, AM, BMD, 6>(splits, a, s); break;
    case 16: launch_glds<64, 64, AM, BMD, 8>(splits, a, s); break;
    case 17: launch_glds<128, 64, AM, BMD, 4>(splits, a, s); break;
    case 18: launch_glds<128, 64, AM, BMD, 6>(splits, a, s); break;
    case 19: launch_glds<64, 64, AM, BMD, 3, 2>(splits, a, s); break;
    case 20: launch_glds<64, 64, AM, BMD, 2, 4>(splits, a, s); break;
    case 21: launch_glds<64, 64, AM, BMD, 4, 2>(splits, a, s); break;
    default: throw std::runtime_error("gemm_dense: bad glds tile id");
  }
}

template <typename T, int AM, int BMD>
static void by_tile(int tile, int splits, const DenseGemmArgs& a, hipStream_t s) {
  switch (tile) {
    case 0: launch_one<T, TileCfg<T, 64, 64, 2, 2, GEMM_KTILE>, AM, BMD>(splits, a, s); break;
    case 1: launch_one<T, TileCfg<T, 128, 128, 2, 2, GEMM_KTILE>, AM, BMD>(splits, a, s); break;
    case 2: launch_one<T, TileCfg<T, 128, 64, 2, 2, GEMM_KTILE>, AM, BMD>(splits, a, s); break;
    case 3: launch_one<T, TileCfg<T, 64, 128, 2, 2, GEMM_KTILE>, AM, BMD>(splits, a, s); break;
    case 4: launch_one<T, TileCfg<T, 32, 32, 2, 2, GEMM_KTILE>, AM, BMD>(splits, a, s); break;
    default: throw std::runtime_error("gemm_dense: bad tile id");
  }
}

template <typename T>
static void by_mode(int am, int bm, int tile, int splits, const DenseGemmArgs& a, hipStream_t s) {
  if (am == KMAJ && bm == KMAJ) by_tile<T, KMAJ, KMAJ>(tile, splits, a, s);
  else if (am == KMAJ && bm == RMAJ) by_tile<T, KMAJ, RMAJ>(tile, splits, a, s);
  else if (am == RMAJ && bm == KMAJ) by_tile<T, RMAJ, KMAJ>(tile, splits, a, s);
  else by_tile<T, RMAJ, RMAJ>(tile, splits, a, s);
}

static bool small_group_record(int amode, int bmode, const DenseGemmArgs& a);

void launch_gemm_dense(int dtype, int amode, int bmode, int tile, int splits, const DenseGemmArgs& args,
                       hipStream_t stream) {
  if (splits < 1) splits = 1;
  if (tile == GEMM_TILE_SMALL) {
    if (!gemm_small_eligible(dtype, args) || splits != 1)
      throw std::runtime_error("gemm_dense: the small-tile kernel takes fp32, one split, no un-pool epilogue");
    if (small_group_record(amode, bmode, args)) return;  // inside a group
    launch_gemm_small(amode, bmode, args, stream);
    return;
  }
  if ((tile == 12 || tile == FC_TILE) && splits == 1 && dtype == 0 && glds_group_record(amode, bmode, tile, args))
    return;  // inside a group
  if (tile == FC_TILE) {
    if (!gemm_fc_eligible(dtype, amode, bmode, args))
      throw std::runtime_error("gemm_dense: this GEMM is not eligible for tile 22 (gemm_fc_eligible)");
    launch_gemm_fc(amode, bmode, splits, args, stream);
    return;
  }
  if (tile >= 5) {
    if (!gemm_glds_eligible(dtype, amode, bmode, tile, args))
      throw std::runtime_error("gemm_dense: this GEMM is not eligible for the global_load_lds tiles");
    if (splits > 1 && !args.atomic && (!args.ws || !args.tile_ctr))
      throw std::runtime_error("gemm_dense: split-K with a fused epilogue needs a workspace");
    if (amode == KMAJ && bmode == KMAJ) glds_by_tile<KMAJ, KMAJ>(tile, splits, args, stream);
    else if (amode == KMAJ && bmode == RMAJ) glds_by_tile<KMAJ, RMAJ>(tile, splits, args, stream);
    else if (amode == RMAJ && bmode == KMAJ) glds_by_tile<RMAJ, KMAJ>(tile, splits, args, stream);
    else glds_by_tile<RMAJ, RMAJ>(tile, splits, args, stream);
    return;
  }
  if (dtype == 0) by_mode<bf16>(amode, bmode, tile, splits, args, stream);
  else by_mode<float>(amode, bmode, tile, splits, args, stream);
}

// ------------------------------------------------------------ grouped launch
// Independent GEMMs of one step phase in ONE launch (horizontal fusion): workgroup ranges of the grid
// run different pieces - the head weight gradient's 257 workgroups (4 columns each), then two 64x64 2-stage glds
// GEMMs (the MNIST-CNN fc1 data and weight gradients).  One launch instead of a fork onto a side
// stream: no cross-queue dependency inside the captured graph (each such edge cost 5-11 us of idle
// time in the step timeline, profiles/r3_cnn_kernel_tuning.txt), and the dispatcher hands out the
// lower workgroup ranges first, so the pieces listed first start first.  Piece ranges are padded to
// multiples of 8 so every piece keeps its own XCD-aware tile order.
struct GlGroupArgs {
  DenseGemmArgs g0, g1;
  HeadWgradArgs h;
  int nh, n0, n1;      // padded workgroup ranges
  int th, t0, t1;      // real workgroups of each piece
};

// HEAD: the head piece is compiled in - the 4-column body (head_wgrad4_body, 40 accumulators per
// thread; the 8-column one set the grouped kernel to ~148 VGPRs against the GEMMs' ~68)
template <int AM0, int BM0, int AM1, int BM1, bool HEAD>
__global__ __launch_bounds__(GEMM_THREADS, 1) void gemm_glds_group_kernel(GlGroupArgs ga) {
  constexpr int HEAD_BYTES = 4 * 40 * 4;
  constexpr int BYTES = GlSmem<64, 64, 2>::BYTES > HEAD_BYTES ? GlSmem<64, 64, 2>::BYTES : HEAD_BYTES;
  __shared__ __attribute__((aligned(16))) char smem_raw[BYTES];
  int bid = blockIdx.x;
  if constexpr (HEAD) {
    if (bid < ga.nh) {
      if (bid < ga.th) head_wgrad4_body<10>(ga.h, bid, reinterpret_cast<float(*)[40]>(smem_raw));
      return;
    }
  }
  bid -= ga.nh;
  if (bid < ga.n0) {
    if (bid < ga.t0) gemm_glds_body<64, 64, AM0, BM0, 2>(ga.g0, bid, smem_raw);
    return;
  }
  bid -= ga.n0;
  if (bid < ga.t1) gemm_glds_body<64, 64, AM1, BM1, 2>(ga.g1, bid, smem_raw);
}

namespace {
struct GlGroupRec {
  bool active = false;
  int tile = 12;  // the pieces' tile: 12 (64x64 glds) or 22 (the 8-wave fc tile, gemm_fc.hip)
  int ng = 0, am[2] = {0, 0}, bm[2] = {0, 0};
  DenseGemmArgs g[2];
  bool has_h = false;
  HeadWgradArgs h;
};
thread_local GlGroupRec g_group;
int pad8(int n) { return (n + 7) / 8 * 8; }
struct SmallGroupRec {  // the fp32 small-tile pieces of the same group (gemm_small.hip)
  int n = 0, am[2] = {0, 0}, bm[2] = {0, 0};
  DenseGemmArgs g[2];
};
thread_local SmallGroupRec g_small;
}  // namespace

static bool small_group_record(int amode, int bmode, const DenseGemmArgs& a) {
  if (!g_group.active || g_small.n == 2) return false;
  g_small.am[g_small.n] = amode;
  g_small.bm[g_small.n] = bmode;
  g_small.g[g_small.n++] = a;
  return true;
}

void glds_group_begin() {
  if (g_group.active) throw std::runtime_error("gemm group: already recording");
  g_group = GlGroupRec();
  g_small = SmallGroupRec();
  g_group.active = true;
}

bool glds_group_record(int amode, int bmode, int tile, const DenseGemmArgs& a) {
  if (!g_group.active || g_group.ng == 2) return false;
  if (g_group.ng == 1 && g_group.tile != tile) return false;
  if (!gemm_glds_eligible(0, amode, bmode, tile, a)) return false;
  g_group.tile = tile;
  g_group.am[g_group.ng] = amode;
  g_group.bm[g_group.ng] = bmode;
  g_group.g[g_group.ng++] = a;
  return true;
}

bool glds_group_record_head(const HeadWgradArgs& a) {
  if (!g_group.active || g_group.has_h || a.B > 1024) return false;
  g_group.has_h = true;
  g_group.h = a;
  return true;
}

void glds_group_end(hipStream_t s) {
  if (!g_group.active) throw std::runtime_error("gemm group: not recording");
  GlGroupRec r = g_group;
  g_group = GlGroupRec();
  const SmallGroupRec sr = g_small;
  g_small = SmallGroupRec();
  if (sr.n) launch_gemm_small_group(sr.n, sr.am, sr.bm, sr.g, s);
  if (r.ng == 0 && !r.has_h) return;
  const bool fused = r.ng == 2 && r.am[0] == KMAJ && r.bm[0] == RMAJ && r.am[1] == RMAJ && r.bm[1] == RMAJ;
  if (!fused) {  // any other combination: the pieces as separate launches, in recording order
    if (r.has_h) launch_head_wgrad(r.h, s);
    for (int i = 0; i < r.ng; ++i) launch_gemm_dense(0, r.am[i], r.bm[i], r.tile, 1, r.g[i], s);
    return;
  }
  if (r.tile == FC_TILE) {
    launch_gemm_fc_group(r.g[0], r.g[1], r.has_h ? &r.h : nullptr, s);
    return;
  }
  GlGroupArgs ga;
  std::memset(&ga, 0, sizeof(ga));
  ga.g0 = r.g[0];
  ga.g1 = r.g[1];
  if (r.has_h) {
    ga.h = r.h;
    ga.th = r.h.K / 4 + (r.h.db ? 1 : 0);
    ga.nh = pad8(ga.th);
  }
  ga.t0 = (ga.g0.M / 64) * ((ga.g0.N + 63) / 64);
  ga.t1 = (ga.g1.M / 64) * ((ga.g1.N + 63) / 64);
  ga.n0 = pad8(ga.t0);
  ga.n1 = ga.t1;
  if (r.has_h)
    hipLaunchKernelGGL((gemm_glds_group_kernel<KMAJ, RMAJ, RMAJ, RMAJ, true>), dim3(ga.nh + ga.n0 + ga.n1),
                       dim3(GEMM_THREADS), 0, s, ga);
  else
    hipLaunchKernelGGL((gemm_glds_group_kernel<KMAJ, RMAJ, RMAJ, RMAJ, false>), dim3(ga.n0 + ga.n1), dim3(GEMM_THREADS),
                       0, s, ga);
}

}  // namespace dtfe
