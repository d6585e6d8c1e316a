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

}  // namespace dtfe
