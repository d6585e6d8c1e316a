#pragma once
#include "common.h"

namespace dtfe {

// MNIST conv1: x [B][28][28] bf16, w [32][5][5] bf16 (cout, kh, kw), bias [32] f32
// fwd : y [B][14][14][32] bf16 pooled ReLU output, argmax [B][14][14][32] u8
// wgrad: dp [B][14][14][32] bf16 pooled gradient (ReLU-masked), argmax -> dw [32][25], db [32] (fp32 +=)
struct Conv1Args {
  int B;
  const bf16* x; const bf16* w; const float* bias;
  bf16* y; uint8_t* argmax;
  const bf16* dp; float* dw; float* db; float scale;
};

void launch_conv1_fwd_pool(const Conv1Args& a, hipStream_t s);
void launch_conv1_wgrad_pooled(const Conv1Args& a, hipStream_t s);

}  // namespace dtfe
