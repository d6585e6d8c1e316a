// Persistent whole-sequence LSTM forward / BPTT.
#pragma once
#include <hip/hip_runtime.h>

#include "elementwise.h"

namespace dtfe {

struct LstmSeqArgs {
  int T, B, I, H;
  float* xh;          // [T][B][I+H]: x_t rows given; h_{t-1} columns of steps 1..T-1 written by the forward
  const float* K;     // [I+H][4H] (TF kernel layout: rows x then h; columns gates i, j, f, o)
  const float* bias;  // [4H]
  float forget_bias;
  float* act;         // [T][B][4H] activated gates (forward out, backward in)
  float* c;           // [T][B][H]
  float* hT;          // [B][H] last hidden state
  const float* dhT;   // [B][H] d loss / d h_T (backward in)
  // optional (backward): dh_T formed in the kernel as dl . W_out^T - dl [B][nc] (the classifier head's
  // dlogits), W_out [H][nc] - instead of read from dhT (one launch and a [B][H] round trip fewer)
  const float* dl; const float* wo; int nc;
  float* dg;          // [T][B][4H] gate pre-activation grads (backward out)
  // optional (forward): st.x != nullptr folds the batch staging (launch_seq_stage: x part of xh, h_{-1} = 0,
  // label copy, accumulator clears) into the forward launch - the split kernel reads x_t straight from the
  // images and writes xh for the kernel gradient in its prologue; other paths stage first
  SeqStageArgs st;
};

// false when the shape is not supported (H != 128, B % 16, (I+H) % 4): callers fall back
bool launch_lstm_seq_fwd(const LstmSeqArgs& a, hipStream_t s);
bool launch_lstm_seq_bwd(const LstmSeqArgs& a, hipStream_t s);

// error word of the split (4 CUs per row group) kernels on the current device: 1 when a
// cross-workgroup exchange timed out since the last reset (the outputs of that launch are
// wrong).  Synchronises the device.  reset clears it.
int lstm_split_status(bool reset);

}  // namespace dtfe

namespace dtfe {
// tall-K exact-fp32 weight gradient (csrc/kernels/wgrad_tallk.hip): out[m][n] = scale * sum_k
// A[k*lda+m] B[k*ldb+n] (stored, m < M), bias[n] = scale * sum_k B[k*ldb+n] (optional)
struct TallKArgs {
  const float* A; int lda;
  const float* B; int ldb;
  int M, N, K;
  float* out; int ldc;
  float* bias;
  float* ws; int splits;
  float scale;
  int MP, kchunk;  // set by the launcher
};
long tallk_ws_floats(int M, int N, int splits);
void launch_wgrad_tallk(const TallKArgs& a, hipStream_t s);
}  // namespace dtfe
