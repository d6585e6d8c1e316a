// Instantiation + dispatch of the dense GEMM kernel family.
#include "gemm_dense.h"
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
  static const int dims[5][2] = {{64, 64}, {128, 128}, {128, 64}, {64, 128}, {32, 32}};
  if (tile < 0 || tile > 4) return -1;
  bm = dims[tile][0];
  bn = dims[tile][1];
  return GEMM_KTILE;
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

void launch_gemm_dense(int dtype, int amode, int bmode, int tile, int splits, const DenseGemmArgs& args,
                       hipStream_t stream) {
  if (splits < 1) splits = 1;
  if (dtype == 0) by_mode<bf16>(amode, bmode, tile, splits, args, stream);
  else by_mode<float>(amode, bmode, tile, splits, args, stream);
}

}  // namespace dtfe
