#pragma once
#include "common.h"

#include <stdexcept>

namespace dtfe {

enum OptKind : int { OPT_SGD = 0, OPT_MOMENTUM = 1, OPT_ADAM = 2, OPT_RMSPROP = 3 };

// A parameter segment of the flat fp32 master buffer.  The segment is viewed
// as [R][T][C]; wt16 (optional) receives the bf16 copy laid out as [C][T][R]
// (dense: W[out][in] -> Wt[in][out]; conv: W[cout][kh*kw][cin] -> Wt[cin][kh*kw][cout]).
struct OptSeg {
  long off;
  int R, T, C;
  bf16* w16;   // natural-layout bf16 working copy (nullable)
  bf16* wt16;  // transposed bf16 working copy (nullable)
};

// Work item: kind 0 = flat range [start, start+count) of segment seg;
// kind 1 = 64x64 tile (r0, c0) of tap t of segment seg (transpose path).
struct OptWork {
  int kind, seg, t, r0, c0;
  long start, count;
};

struct OptArgs {
  int kind;
  float* p;
  const float* g; const bf16* g16; float gscale;   // exactly one of g / g16
  float* s1; float* s2;                            // slots (adam: m, v; rmsprop: ms, mom; momentum: accum)
  float lr, beta1, beta2, eps, momentum, rho;
  float* beta_pow;          // adam: [beta1_power, beta2_power] (TF1 non-slot variables)
  int32_t* global_step; int gs_inc;
  uint32_t* done_counter;   // zero-initialised; reset by the last workgroup
  const OptSeg* segs; const OptWork* work; int nwork;
};

void launch_apply_gradients(const OptArgs& a, hipStream_t s);

// up to OPT_GROUP_MAX optimizers of one kind in a single launch (contiguous workgroup ranges)
constexpr int OPT_GROUP_MAX = 4;
struct OptGroup {
  OptArgs o[OPT_GROUP_MAX];
  int first[OPT_GROUP_MAX + 1];
  int n;
};
void launch_apply_gradients_group(const OptArgs* o, int n, hipStream_t s);

}  // namespace dtfe
