// 8-wave 256x128 bf16 GEMM with direct global->LDS staging (tile 22 of launch_gemm_dense): the
// MNIST-CNN fc1 GEMMs (M, N in {1024, 3136(+1)}, K in {1024, 3136}).
//
// Why a second glds family: the fc1 GEMMs are bound by the per-CU L2 -> LDS stream, not by MFMA
// (a 64x64 tile moves (64 + 64) * K * 2 bytes for 64 * 64 * K * 2 FLOP: 32 FLOP/B).  One 256x128
// tile per CU moves 85 FLOP/B, so the fc1 data + weight gradients need 154 MB of L2 -> LDS traffic
// instead of 410 MB with 64x64 tiles; 8 waves (4 x 2 wave grid, 64 x 64 per wave, 16 accumulators)
// keep 6 DMA pieces per thread in flight per k-tile.  N need not be a multiple of 128: the last
// n-tile clamps its source columns inside the row (outputs past N are never stored) and the bias
// column of a weight-gradient GEMM (b_ones_row = N - 1) reads a page of ones.
#pragma once
#include "gemm_dense.h"
#include "head.h"

namespace dtfe {

constexpr int FC_TILE = 22;
constexpr int FC_BM = 256, FC_BN = 128, FC_THREADS = 512;

// whether tile 22 can run this GEMM (bf16, M % 256 == 0, K % 64 == 0, 16 B aligned operands; a
// KMAJ B operand needs whole n-tiles)
bool gemm_fc_eligible(int dtype, int amode, int bmode, const DenseGemmArgs& a);
void launch_gemm_fc(int amode, int bmode, int splits, const DenseGemmArgs& a, hipStream_t s);
// the grouped fc backward: head weight gradient (optional) + a (KMAJ, RMAJ) and a (RMAJ, RMAJ) GEMM
void launch_gemm_fc_group(const DenseGemmArgs& g0, const DenseGemmArgs& g1, const HeadWgradArgs* h, hipStream_t s);

}  // namespace dtfe
