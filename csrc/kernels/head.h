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
  // optional: advanced by one (one thread of workgroup 0) - the per-step sampling / dropout
  // counter of the fused MNIST step, whose readers (the conv1 gather, fc1 dropout) all run
  // before this kernel: one plain increment instead of a grid-wide last-arriver atomic
  int64_t* step_counter;
};

void launch_head_xent(const HeadArgs& a, hipStream_t s);

// dW[c][k] = scale * sum_b dl[b][c] h[b][k] (row stride ldw), db[c] = scale * sum_b dl[b][c];
// stored, not accumulated (one workgroup per 16 columns, fixed summation order)
struct HeadWgradArgs {
  int B, NC, K;
  const bf16* dl; int ld_dl;   // [B][ld_dl]
  const bf16* h; int ldh;      // [B][ldh]
  float* dw; int ldw;          // [NC][ldw]
  float* db;                   // [NC] (optional)
  float scale;
};
void launch_head_wgrad(const HeadWgradArgs& a, hipStream_t s);

}  // namespace dtfe
