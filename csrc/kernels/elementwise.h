#pragma once
#include "common.h"

namespace dtfe {

// ---- data path: HBM-resident dataset -> batch
// src dtype: 0 = uint8 (raw pixels, scaled by 1/255), 1 = f32, 2 = bf16
// dst dtype: 1 = f32, 2 = bf16
// idx == nullptr: indices sampled on device from (seed, *counter) and the
// counter advanced by the last workgroup, so a replayed graph draws a new batch.
struct GatherArgs {
  const void* src; int src_dtype; long n_rows; int D;
  void* dst; int dst_dtype; int B;
  const int32_t* idx;
  const int32_t* labels_src; int32_t* labels_dst;
  uint64_t seed; int64_t* counter; uint32_t* done;
  // step-prologue zeroing fused into the same launch: up to 4 word ranges (accumulators the
  // step's atomics add into - loss / hit counters, atomically reduced weight grads)
  uint32_t* zptr[4]; long zlen[4]; int nz;
  // optional one-hot label rows [B][ncls] fp32 written in the same launch (softmax-xent input)
  float* onehot; int ncls;
};
void launch_gather_rows(const GatherArgs& a, hipStream_t s);

// uniform noise U(lo, hi) from a counter-based hash; *counter advanced per call
void launch_uniform_fill(float* out, long n, float lo, float hi, uint64_t seed, int64_t* counter,
                         uint32_t* done, hipStream_t s, const float* csrc = nullptr, float* cdst = nullptr,
                         long ncopy = 0);

// LSTM batch staging in ONE launch (reference lstm/distributed_lstm.py:127 reshape): image rows
// x[B][T][I] -> the x part of the per-step [x_t, h_{t-1}] rows xh[T][B][ld] (ld = I + H), the h_{-1}
// part of step 0 zeroed, ny label floats copied, up to 4 word ranges (loss / hit accumulators)
// cleared.
struct SeqStageArgs {
  const float* x; float* xh; int B, T, I, ld;
  const float* ysrc; float* ydst; long ny;
  uint32_t* zptr[4]; long zlen[4]; int nz;
};
void launch_seq_stage(const SeqStageArgs& a, hipStream_t s);

// dtype casts
void launch_cast_f32_bf16(const float* src, bf16* dst, long n, hipStream_t s);
void launch_cast_bf16_f32(const bf16* src, float* dst, long n, hipStream_t s);

// softmax cross-entropy fwd+bwd on fp32 logits [B][NC]
// labels: int32 class ids (labels_i) or one-hot fp32 rows (labels_oh).
// dlogits = (softmax - y) * scale; loss_rows[b] = per-row loss; correct += argmax hits
struct XentArgs {
  int B, NC;
  const float* logits; const int32_t* labels_i; const float* labels_oh;
  float scale;
  float* dlogits; float* loss_rows; float* loss_sum; int32_t* correct; float* probs;
};
void launch_softmax_xent(const XentArgs& a, hipStream_t s);

// A small dense classifier head, forward AND backward, in ONE workgroup (ResNet-20: 64 features ->
// 10 classes, B = 256): logits = feat W^T + b (fp32, also stored), softmax cross-entropy against
// one-hot labels (loss sum += , hit count +=), dlogits = (p - y) scale, dW += dlogits^T feat,
// db += column sums of dlogits, dfeat = bf16(dlogits W).  Replaces the cast / GEMM / softmax /
// GEMM / column-sum / GEMM / cast chain (7 launches).  False when it does not fit one workgroup's LDS.
struct DenseHeadArgs {
  const void* feat; const float* w; const float* bias; const float* y;  // [B][F], [NC][F], [NC], [B][NC]
  float* logits; float* loss_sum; int32_t* correct;
  float* dw; float* db; void* dfeat;                                    // [NC][F] +=, [NC] +=, [B][F]
  int B, F, NC; float scale;
  int f32;       // feat / dfeat are fp32 (else bf16)
  int w_fmajor;  // W (and dW) stored [F][NC] (a TF Variable of shape (in, out)) instead of [NC][F]
  int store;     // dW / db are stored, not accumulated
  int slices;    // (set by the launcher) batch slices of the dW phase
  int ylds;      // (set by the launcher) the labels are staged in LDS (when they fit)
  float* dl_out; // optional: the dlogits rows [B][NC] (fp32) - the consumer forms dfeat itself (dfeat may then be null)
  int diag;      // (set by the launcher) DTFE_DIAG dh=<bits> phase-skipping ablation: 1 logits, 2 softmax,
                 // 4 dW, 8 dfeat, 16 db, 32 feature staging - timing only, never for training
};
bool launch_dense_head(const DenseHeadArgs& a, hipStream_t s);

// GAN losses on the sigmoid outputs of D, with grads w.r.t. the
// pre-sigmoid logits.  No epsilon inside log, as in the reference (GAN:142-143),
// unless clamp_eps > 0.
struct GanLossArgs {
  int B;
  const float* d_real; const float* d_fake;   // sigmoid outputs [B]
  float* gen_loss; float* disc_loss;          // scalars (overwritten)
  float* dz_real_disc; float* dz_fake_disc;   // d disc_loss / d logit
  float* dz_fake_gen;                         // d gen_loss / d logit_fake
  float clamp_eps;
};
void launch_gan_loss(const GanLossArgs& a, hipStream_t s);

// mean((t - y)^2) with the gradient w.r.t. the pre-sigmoid logit of y.  ws (optional,
// MSE_WS_FLOATS floats, zeroed once): the loss is stored by the last workgroup (no memset, deterministic)
constexpr int MSE_PARTS = 128;
constexpr int MSE_WS_FLOATS = MSE_PARTS + 4;
void launch_mse_sigmoid(const float* y, const float* t, long n, float* loss, float* dz, hipStream_t s,
                        float* ws = nullptr);

// db[n] += scale * sum_m x[m][n]   (x f32 or bf16)
void launch_colsum(const void* x, int x_f32, int M, int N, long ld, float* db, float scale, hipStream_t s);

// dz = dy * act'(y)   (y = forward output of the activation)
void launch_act_grad(const float* dy, const float* y, float* dz, long n, int act, hipStream_t s);

// out = act(x + bias[col]) ; optional dropout (keep prob, hash RNG) ; bf16 or f32 out
struct BiasActArgs {
  const float* x; const float* bias; int M, N; int act;
  float keep; uint64_t seed; const int64_t* counter;
  void* out; int out_f32;
};
void launch_bias_act(const BiasActArgs& a, hipStream_t s);

// TF BasicLSTMCell (gate order i, j, f, o; forget_bias added to f) - SURVEY K05/K06.
// fwd:  gates [B][4H] pre-activations (incl. bias) -> act [B][4H] (sigmoid i, tanh j,
//       sigmoid f+fb, sigmoid o), c [B][H], h written to h_out (row stride ld_h).
// bwd:  dh [B][H] (+ dh2 optional), dc_next [B][H] -> dgates [B][4H] (pre-activation),
//       dc_prev [B][H] (may alias dc_next).
struct LstmCellArgs {
  int B, H;
  const float* gates; float* act; const float* c_prev; float* c; float* h_out; long ld_h;
  const float* dh; const float* dh2; const float* dc_next; float* dgates; float* dc_prev;
  float forget_bias;
};
void launch_lstm_cell_fwd(const LstmCellArgs& a, hipStream_t s);
void launch_lstm_cell_bwd(const LstmCellArgs& a, hipStream_t s);

}  // namespace dtfe
