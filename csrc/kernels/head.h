#pragma once
#include "common.h"
#include <stdexcept>

namespace dtfe {

struct HeadArgs {
  int B, NC, K;
  const bf16* h; const bf16* w; const float* b; const int32_t* labels;
  float scale;        // d(loss)/d(logit) scale: 1 / batch
  float inv_keep;     // dropout scale of h (1 when no dropout)
  bf16* dz;           // [B][K]
  bf16* dl; int ld_dl;  // d(loss)/d(logit) rows, bf16 [B][ld_dl]
  float* loss_sum; int32_t* correct; float* logits_out;
};

void launch_head_xent(const HeadArgs& a, hipStream_t s);

}  // namespace dtfe
