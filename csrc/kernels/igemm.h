// Implicit-GEMM convolution for wide NHWC layers (C % 64 == 0, Cout % 64 == 0):
// the ResNet-50 bottleneck / projection convs.  Operands are staged into LDS with
// gfx950's direct global->LDS DMA (global_load_lds_dwordx4) in 64-deep k-tiles;
// out-of-image taps read a zero page, so the main loop has no per-element branches.
//
//   forward   rows = output pixels, k = (tap, cin), B = W[cout][tap][cin]
//   dgrad     the same kernel over dY with Wt[cin][tap][cout], one launch phase per
//             output-pixel parity class (py, px) of a strided conv: phase p only
//             visits the taps that reach its pixels (sub-pixel decomposition), so a
//             stride-2 data gradient does no multiply-by-zero work
//   wgrad     dW[cout][tap][cin] = sum_m dY[m][cout] X[src(m, tap)][cin]; the m
//             reduction is split over workgroups, partial tiles go to a workspace
//             and one reduce pass adds them (scaled) into the fp32 gradient.
#pragma once
#include "common.h"
#include "conv.h"

namespace dtfe {

constexpr int IG_MAX_TAPS = 9;

// One launch phase: rows are the pixels (b, i, j) of a RH x RW grid, written to
// output pixel (i*ostr + oy, j*ostr + ox); tap t reads source pixel
// (i*istr + dy[t], j*istr + dx[t]) and weight tap kt[t].
struct IgPhase {
  int ntaps, RH, RW, oy, ox;
  int dy[IG_MAX_TAPS], dx[IG_MAX_TAPS], kt[IG_MAX_TAPS];
};

struct IgemmArgs {
  const bf16* src; const bf16* w; bf16* out; float* ws; const bf16* zeros;
  int B, SH, SW, SC;      // source tensor (NHWC)
  int N, Ktot;            // output channels; weight row length = taps * SC
  int istr, OHf, OWf, ostr;
  int nphase, splits, tiles_m;
  int accum;              // out += result (bf16 read-modify-write in the epilogue)
  // accum with a masked source: out = result + acc_src * bit (acc_mask: 1-bit [rows][N/8] mask at the
  // output's pixel / channel), read instead of out - a residual block's shortcut gradient
  // (dout * ReLU'(block output)) added where the input gradient is produced, never stored alone
  const bf16* acc_src; const uint8_t* acc_mask;
  // forward only: per output tile and channel the BatchNorm partials of the stored (bf16) output,
  // [tiles_m][3][N] = (K_t = the tile's first row, sum (y - K_t), sum (y - K_t)^2)
  float* bn_part;
  // data gradient only (bb_x != nullptr): BatchNorm-backward statistics of the stored (final) output
  // for the BN that consumes it, g = out * act'(.), into bn_part as (0, sum g, sum g*xhat) per tile
  // (tile index = phase * tiles_m + tm; zero shift, so the forward reduce kernels fold them as is).
  // bb_y == nullptr with ReLU: the mask is recomputed from x (norm.hip BwdMask).
  const bf16* bb_x; const bf16* bb_y; const float* bb_mean; const float* bb_invstd;
  const float* bb_gamma; const float* bb_beta; int bb_act;
  IgPhase ph[4];
};

struct IgWgradArgs {
  const bf16* dy; const bf16* x; const bf16* zeros; float* ws;
  int B, H, W, C, OH, OW, Cout, KH, KW, stride, pad;
  int splits, mchunk;
};

// BatchNorm statistics from per-tile shifted partials (any producer's epilogue): part holds
// [tiles][3][N] = (K_t = the tile's first row, sum (y - K_t), sum (y - K_t)^2) of tiles of BMr rows
// (the last one Mp - (tiles-1)*BMr); two fixed-order fold launches add (sum, sumsq) around row 0's
// value into stats[2][N], as bn_stats would.  bn_part_buffer: the device scratch for `tiles`
// tiles plus the fold's chunk table (valid until the next call on this device).
float* bn_part_buffer(long tiles, int N, hipStream_t s);
// a zeroed hand-off counter beside a bn_part_buffer (not one the fold launches use); whoever takes
// it leaves it zero again (last-arriver reset)
uint32_t* bn_part_counter(const float* part);
void launch_bn_part_reduce(float* part, int tiles, int N, long Mp, int BMr, float* stats, hipStream_t s);

// true when the igemm path handles the conv (and launches it)
// stats_done (optional): set when f.bn_stats was produced by the fused epilogue partials
bool launch_igemm_fwd(const ConvFwdArgs& a, hipStream_t s, bool* stats_done = nullptr);
bool launch_igemm_dgrad(const ConvDgradArgs& a, hipStream_t s);
bool launch_igemm_wgrad(const ConvWgradArgs& a, hipStream_t s);

}  // namespace dtfe
