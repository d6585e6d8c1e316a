// Exact-fp32 NHWC convolution launchers (conv_f32.hip): the `--dtype fp32` MNIST CNN step.
#pragma once
#include "conv.h"

namespace dtfe {

struct ConvF32Args {
  ConvGeom g;            // g.pool_order: forward rows in 2x2 pool-window order (fused max-pool)
  const float* src;      // fwd: x [B][H][W][C]; dgrad: dY [B][OH][OW][Cout]; wgrad: dZ [B*OH*OW][Cout]
  const float* w;        // fwd: W [Cout][KH][KW][C]; dgrad: Wt [C][KH][KW][Cout]
  const float* x;        // wgrad: the forward input
  const float* bias;     // fwd (optional)
  float* out;            // fwd: y (pooled when pool_order); dgrad: dX
  uint8_t* argmax;       // fwd + pool (optional): 0..3 = dy * 2 + dx of the window's maximum
  const float* relu_mask;  // dgrad (optional): dX = mask > 0 ? dX : 0
  float* dw; float* db;  // wgrad: dW += scale * ..., db += scale * ... (optional)
  float scale;
  int act;
  int k_chunk;
};

void launch_conv_fwd_f32(const ConvF32Args& a, hipStream_t s);
void launch_conv_dgrad_f32(const ConvF32Args& a, hipStream_t s);   // stride 1
void launch_conv_wgrad_f32(const ConvF32Args& a, hipStream_t s);
void launch_unpool_f32(const float* g, const uint8_t* am, float* out, int B, int PH, int PW, int C, hipStream_t s);
void launch_transpose_taps_f32(const float* in, float* out, int O, int T, int C, hipStream_t s);
// MNIST conv1's weight gradient (C = 1, 32 channels, 3x3 / 5x5 SAME, stride 1) straight from the pooled
// gradient dP [B][H/2][W/2][32] and its argmax bytes: dW += scale * sum, db += scale * sum over the
// non-zero (argmax) pixels only, through ws (>= conv1_wgrad_pooled_f32_ws_floats(B) floats) and a
// fixed-order partial reduce.  false: shape not covered (un-pool + launch_conv_wgrad_f32 instead).
long conv1_wgrad_pooled_f32_ws_floats(int B);
bool launch_conv1_wgrad_pooled_f32(const float* dp, const uint8_t* am, const float* x, float* dw, float* db, float* ws,
                                   long ws_floats, const ConvGeom& g, float scale, hipStream_t s);

}  // namespace dtfe
