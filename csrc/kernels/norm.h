#pragma once
#include "common.h"

namespace dtfe {

// BatchNorm (training mode) over NHWC bf16 activations viewed as [R = B*H*W][C]
// (C % 8 == 0), plus the residual-shortcut and pooling pieces of a ResNet block.
//
// Forward:   stats += (sum d, sum d^2), d = x - x[row 0]        (bn_stats, atomics into a zeroed [2][C])
//            y = act(gamma * (x - mean) * invstd + beta + shortcut(res))   (bn_apply)
//            the apply launch also stores mean / invstd and updates the moving averages
// Backward:  g = dy * act'(y);  stats += (sum g, sum g * xhat)  (bn_bwd_stats)
//            dx = gamma * invstd * (g - sum g / R - xhat * sum(g xhat) / R)   (bn_bwd_apply)
//            dgamma += sum(g xhat), dbeta += sum g; optional dres = g (shortcut gradient)
//
// Shortcut modes (ResNet v1 "option A" identity): the residual tensor has
// (RH, RW, RC) and is read at (y*rstride, x*rstride, c) for c < RC, zero for
// the extra channels of a widening block.
struct BnArgs {
  long R; int C;
  const bf16* x;                 // [R][C] pre-normalisation input (conv output)
  const bf16* y;                 // forward output (backward: ReLU mask source)
  const bf16* dy;                // backward: upstream gradient [R][C]
  float* stats;                  // [2][C] accumulators (zeroed by the caller)
  const float* gamma; const float* beta;
  float* mean; float* invstd;    // saved batch statistics [C]
  float* moving_mean; float* moving_var;
  float eps, momentum;           // TF: moving = moving * momentum + batch * (1 - momentum)
  int act;
  // residual (forward add / backward copy of the masked gradient)
  const bf16* res; bf16* dres; int RH, RW, RC, rstride, OH, OW;
  bf16* out;                     // forward y / backward dx
  float* dgamma; float* dbeta;   // backward parameter gradients (+=)
  int infer;                     // bn_apply only: normalise with the moving averages (inference mode;
                                 // stats unused, nothing is updated or saved)
  // 1-bit ReLU mask [R][C/8] bytes (bit e of byte (r, c/8) = out[r][c] > 0, c = 8 * (c/8) + e):
  // bn_apply writes it (mask_out) beside a ReLU output that had a residual added; the backward
  // kernels read it (ymask) instead of that bf16 output - 1 byte per 8 channels instead of 16
  uint8_t* mask_out;
  const uint8_t* ymask;
  // bn_apply only: the residual through its own BatchNorm (a projection shortcut, no activation).
  // res is then the shortcut conv's RAW output (same shape as x); its batch statistics r_stats
  // (accumulated like stats), r_gamma / r_beta normalise it on the fly - rounded to bf16 exactly as
  // bn_apply would have stored that BN's output - and workgroup 0 also saves r_mean / r_invstd and
  // updates r_moving_mean / r_moving_var.  The shortcut BN's own apply pass (write + re-read of its
  // output) disappears.
  // bn_bwd_stats only (MM_BITS): res = that projection BN's input; r_mean / r_invstd its saved batch
  // statistics, and its backward statistics (sum g, sum g * xhat_res) are accumulated into r_stats
  // from the same g in the same pass (g = dy * the block output's ReLU bit)
  float* r_stats; const float* r_gamma; const float* r_beta;
  float* r_mean; float* r_invstd; float* r_moving_mean; float* r_moving_var;
};

void launch_bn_stats(const BnArgs& a, hipStream_t s);
void launch_bn_apply(const BnArgs& a, hipStream_t s);
void launch_bn_bwd_stats(const BnArgs& a, hipStream_t s);
void launch_bn_bwd_apply(const BnArgs& a, hipStream_t s);

// dx[b, y*stride, x*stride, c] += g[b, y, x, c] for c < XC (option-A shortcut gradient)
void launch_shortcut_grad_add(const bf16* g, bf16* dx, int B, int OH, int OW, int C, int XH, int XW, int XC,
                              int stride, hipStream_t s);

// global average pool: x [B][HW][C] -> y [B][C] (bf16), and its backward
void launch_gap_fwd(const bf16* x, bf16* y, int B, int HW, int C, hipStream_t s);
void launch_gap_bwd(const bf16* dy, bf16* dx, int B, int HW, int C, hipStream_t s);

// 3x3/stride-2/pad-1 max pool (ResNet-50 stem) with argmax (0..8), and its backward
void launch_maxpool3_fwd(const bf16* x, bf16* y, uint8_t* am, int B, int H, int W, int C, int OH, int OW,
                         hipStream_t s);
void launch_maxpool3_bwd(const bf16* dy, const uint8_t* am, bf16* dx, int B, int H, int W, int C, int OH, int OW,
                         hipStream_t s);
// maxpool3_bwd fused into the following BatchNorm's backward (ReLU mask from x): a.dy = the POOLED
// gradient [B][OH][OW][C], am its argmax, a.x the BN input [B][H][W][C]; launches the statistics
// pass (into a.stats, zeroed by the caller) and the apply pass (a.out = dx, dgamma / dbeta +=)
void launch_pool3_bn_bwd(const BnArgs& a, const uint8_t* am, int B, int H, int W, int OH, int OW, hipStream_t s);
// bn_apply (training mode, ReLU) fused with maxpool3_fwd: x = the conv output [B][H][W][C] (a.x,
// a.stats, gamma, beta, mean / invstd / moving averages as bn_apply) -> pooled y + argmax; the
// normalised map is never stored (ResNet-50 stem)
void launch_bn_relu_pool3(const BnArgs& a, bf16* y, uint8_t* am, int B, int H, int W, int OH, int OW,
                          hipStream_t s);

}  // namespace dtfe
