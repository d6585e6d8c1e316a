// Convolution / pooling argument blocks shared by the kernels and the bindings.
#pragma once
#include "common.h"

namespace dtfe {

struct ConvGeom {
  int B, H, W, C;          // input NHWC
  int Cout, OH, OW;        // output
  int KH, KW, stride, pad;
  int pool_order;          // forward rows enumerated by 2x2 pool window (fused max-pool)
};

// Un-pool description: the GEMM output element at flat index pidx of a pooled
// tensor [B, PH, PW, C] is a gradient w.r.t. pooled value P[pidx]; it is routed
// to position argmax[pidx] of its 2x2 window in the full-resolution tensor
// [B, 2PH, 2PW, C] (zeros elsewhere) and masked by ReLU'(P) (P > 0).
struct UnpoolArgs {
  const bf16* pooled;
  const uint8_t* argmax;
  int PH, PW, C;
};

__device__ __forceinline__ void unpool_store(const UnpoolArgs& u, long pidx, float g, bf16* dz) {
  const int c = (int)(pidx % u.C);
  long t = pidx / u.C;
  const int pw = (int)(t % u.PW);
  t /= u.PW;
  const int ph = (int)(t % u.PH);
  const long b = t / u.PH;
  const int am = u.argmax[pidx];
  const float gv = bf2f(u.pooled[pidx]) > 0.f ? g : 0.f;
  const int W2 = 2 * u.PW, H2 = 2 * u.PH;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const long o = ((b * H2 + 2 * ph + (q >> 1)) * W2 + 2 * pw + (q & 1)) * u.C + c;
    dz[o] = f2bf(q == am ? gv : 0.f);
  }
}

struct ConvFwdArgs {
  ConvGeom g;
  const bf16* x; const bf16* w; const float* bias;
  bf16* y; uint8_t* argmax; int act;
  float* bn_stats;   // optional [2][Cout] (zeroed): BatchNorm statistics of y, as bn_stats computes them
};
struct ConvDgradArgs {
  ConvGeom g;
  const bf16* dy; const bf16* wt;   // wt: [C][KH][KW][Cout]
  bf16* dx; int unpool; UnpoolArgs up;
  const bf16* relu_mask;            // optional: dx = mask > 0 ? dx : 0 (ReLU' of a pooled output)
  int accumulate;                   // dx += dgrad (implicit-GEMM path only)
  // optional (bnb_stats != nullptr): the consuming BatchNorm's backward statistics of the final dx,
  // bnb_stats += (sum g, sum g*xhat), g = dx * act'(.) (norm.h launch_bn_bwd_stats semantics) -
  // from the implicit-GEMM epilogue where it can, else a separate statistics pass
  const bf16* bnb_x; const bf16* bnb_y; const float* bnb_mean; const float* bnb_invstd;
  const float* bnb_gamma; const float* bnb_beta; float* bnb_stats; int bnb_act;
  const uint8_t* bnb_ymask;   // 1-bit ReLU mask instead of bnb_y (norm.h BnArgs::ymask)
  // accumulate onto acc_src * mask instead of onto dx's contents (igemm.h IgemmArgs::acc_src)
  const bf16* acc_src; const uint8_t* acc_mask;
};
struct ConvWgradArgs {
  ConvGeom g;
  const bf16* dz; const bf16* x;    // dz: [B*OH*OW][Cout] (full resolution)
  float* dw; float* db; float scale; int k_chunk;
};

void launch_conv_fwd(const ConvFwdArgs& a, hipStream_t s);
// the separate BN-backward statistics pass over a finished dx (ConvDgradArgs::bnb_*)
void launch_dgrad_bn_bwd_stats(const ConvDgradArgs& a, hipStream_t s);
// dedicated ImageNet stem (7x7/2, 3 -> 64, 224 -> 112; stem.hip): true when it handled the call
bool launch_stem_fwd(const ConvFwdArgs& a, hipStream_t s, bool* stats_done = nullptr);
bool launch_stem_wgrad(const ConvWgradArgs& a, hipStream_t s, bool accumulate);
void launch_conv_dgrad(const ConvDgradArgs& a, hipStream_t s);
void launch_conv_wgrad(const ConvWgradArgs& a, hipStream_t s);

}  // namespace dtfe
