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
  // second destinations of the updated values (nullable): a ps writes the requesting worker's
  // reply buffer from the apply itself - bf16 natural / transposed copies, or the fp32 value of
  // a variable without bf16 copies - instead of snapshotting its working copies afterwards
  bf16* w16b;
  bf16* wt16b;
  float* pb;
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
  int skip_advance;         // 1: leave the beta powers / global step alone (a partial apply: the
                            // ps applies a push bucket by bucket, then launch_opt_advance once)
  // ps reply folded into the launch (rep_slot != nullptr): after every workgroup's stores have
  // completed, the last one publishes (global step, version, stale, seq) into the worker's slot
  // of the shared page (ps_link.h), exactly as ps_reply_kernel would after this launch
  uint64_t* rep_slot;
  const int32_t* rep_gs;
  uint64_t rep_seq, rep_ver;
  int rep_stale;
  // optional device-side dependency (a gradient produced on another stream with no graph edge to this
  // launch): the work items of segments in wait_segs wait until *wait_done exceeds *wait_seen (set by
  // epoch_signal_kernel after the producer); the last workgroup then advances *wait_seen
  const int* wait_done; int* wait_seen; uint32_t wait_segs;
};
// *ctr += 1 (agent-scope release) - launched on the producer's stream right after the producer
void launch_epoch_signal(int* ctr, hipStream_t s);

void launch_apply_gradients(const OptArgs& a, hipStream_t s);
// the non-slot scalars of one optimizer step: beta powers (Adam) and global_step += gs_inc
void launch_opt_advance(const OptArgs& a, hipStream_t s);
// the step scalars of n (<= OPT_GROUP_MAX) optimizers and then, if a[n-1].rep_slot is set, its
// reply words - one launch (a ps request whose gradient was all applied bucket by bucket)
void launch_opt_advance_reply(const OptArgs* a, int n, hipStream_t s);

// TF1 Adam step of one element: m = b1 m + (1-b1) g; v2 = b2 v2 + (1-b2) g^2; p -= lr_t m / (sqrt(v2) + eps).
// No multiply-add contraction: the rounding must not depend on a kernel's instruction selection.
__device__ __forceinline__ float tf1_adam(float p, float g, float& m, float& v2, float lr_t, float beta1, float beta2,
                                          float eps) {
#pragma clang fp contract(off)
  m = m * beta1 + (1.f - beta1) * g;
  v2 = v2 * beta2 + (1.f - beta2) * g * g;
  return p - lr_t * m / (sqrtf(v2) + eps);
}
__device__ __forceinline__ float tf1_adam_lr(float lr, const float* beta_pow) {
#pragma clang fp contract(off)
  return lr * sqrtf(1.f - beta_pow[1]) / (1.f - beta_pow[0]);
}

// up to OPT_GROUP_MAX optimizers of one kind in a single launch (contiguous workgroup ranges)
constexpr int OPT_GROUP_MAX = 4;
struct OptGroup {
  OptArgs o[OPT_GROUP_MAX];
  int first[OPT_GROUP_MAX + 1];
  int n;
};
void launch_apply_gradients_group(const OptArgs* o, int n, hipStream_t s);

}  // namespace dtfe
