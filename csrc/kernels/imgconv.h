#pragma once
#include "bn_chan.h"
#include "common.h"

namespace dtfe {

// Whole-image implicit-GEMM convolution for small feature maps (MNIST 14x14,
// CIFAR 32x32 ... 8x8): one workgroup stages a complete zero-padded NHWC image
// in LDS and builds every MFMA A fragment straight from it (one ds_read_b128
// of 8 channels at pixel + tap), instead of re-reading the 25x im2col
// expansion from L2 for every k-step.  The weights stream through registers
// (16-byte fragment loads, L2-resident).
//
// Forward:  y[p][n] = sum_{tap,c} src[p*stride - pad + tap][c] * w[n][tap][c]
// CS == 1 (the network input) uses a tap-packed variant: k = tap (<= 32).
// Data-grad (stride 1): the same loop over dY with pad' = K-1-pad and the taps
// of Wt[n=cin][tap][c=cout] flipped (flip_taps = 1).
// Optional on-load un-pool of the source (src = unpool(src_pooled, src_argmax)),
// and epilogues: +bias, activation, 2x2 max-pool + argmax (rows in pool order),
// ReLU mask of a pooled tensor (dgrad), plain store.
struct ImgConvArgs {
  int B, SH, SW, CS;        // source image (per batch element) [SH][SW][CS]
  int OH, OW, N;            // output pixels and channels
  int KH, KW, stride, pad;
  int flip_taps;
  int dil;                  // source dilation (0/1: none): source pixel (y, x) sits at (y*dil, x*dil)
                            // of the zero-padded image - the data gradient of a strided conv
  const bf16* src;          // [B][SH][SW][CS]   (or nullptr with src_pooled)
  const bf16* src_pooled;   // [B][SH/2][SW/2][CS] pooled values to route through src_argmax
  const uint8_t* src_argmax;
  const bf16* w;            // [N][KH*KW][CS]
  const float* bias;
  int act, pool;
  bf16* y;                  // [B][OH'][OW'][N]  (OH' = OH/2 when pooling)
  uint8_t* argmax;          // pool argmax out (optional)
  const bf16* relu_mask;    // dgrad epilogue: y = mask > 0 ? y : 0 (same indexing as y)
  // optional batch sampling fused into the network-input conv (MNIST conv1 forward): image b is
  // row hash(g_seed, step * B + b) % g_rows of the HBM-resident uint8 dataset g_src (step =
  // *g_counter, advanced by the last workgroup), converted to bf16 on load and also stored to
  // src (the weight gradient's input) with its label; zptr/zlen: the step's accumulators,
  // cleared by the same launch (replaces the separate gather kernel of the step)
  const uint8_t* g_src;
  long g_rows;
  uint64_t g_seed;
  int64_t* g_counter;
  uint32_t* g_done;
  const int32_t* g_labels_src;
  int32_t* g_labels_dst;
  uint32_t* zptr[4];
  long zlen[4];
  int nz;
  int diag;                 // ablation bits for kernel experiments (DTFE_DIAG ic=<bits>; 0 in production)
  // diagnostics (bench/resnet20_kernels.py --phases): per-workgroup s_memrealtime stamps [grid][8] at the
  // persistent kernel's phase boundaries, written by thread 0 (nullptr in production)
  uint64_t* tstamp;
  // option-A shortcut gradient added in the (LDS-staged) epilogue of a data gradient:
  // y[b][oy][ox][c] += sc_src[b][oy/s][ox/s][c] where oy, ox are multiples of s = sc_stride
  // (sc_src: [B][OH/s][OW/s][sc_C], c < N <= sc_C) - ops.shortcut_grad_add without its pass
  const bf16* sc_src;
  int sc_stride, sc_C;
  // BatchNorm + ReLU of the source formed while staging it (persistent kernel, plain source; the
  // source is the BN's raw input).  bns.stats == nullptr: none
  BnSrc bns;
};

// Whole-image weight gradient:  dW[n][tap][c] += sum_p dY[p][n] * src[p*stride - pad + tap][c]
// (+ db[n] += sum_p dY[p][n]); dY optionally un-pooled on load from (dy_pooled, dy_argmax).
// CS == 1 uses a tap-packed variant (dW^T = shifted-image^T x dY, <= 32 taps).
struct ImgWgradArgs {
  int B, SH, SW, CS, OH, OW, N, KH, KW, stride, pad;
  const bf16* src;                                   // [B][SH][SW][CS]
  const bf16* dy;                                    // [B][OH][OW][N]  or nullptr with dy_pooled
  const bf16* dy_pooled; const uint8_t* dy_argmax;   // [B][OH/2][OW/2][N]
  float* dw; float* db; float scale;
  int imgs_per_block;
  // optional partial-sum workspace for the persistent kernel, >= 256 * (N*KH*KW*CS + N) floats:
  // per-workgroup partials are stored plainly and summed by a second kernel (cheaper than
  // 256-way contended fp32 atomics on every dW element); null -> atomics
  float* ws;
  // persistent-kernel grid cap (0: 256 = one workgroup per CU).  Fewer workgroups accumulate
  // more images each and halve the partial-sum traffic - the better trade when the launch
  // runs beside other work (MNIST conv2's weight grad on its own graph branch)
  int max_blocks;
  int diag;                 // ablation bits for kernel experiments (DTFE_DIAG iw=<bits>; 0 in production)
  BnSrc bns;                // BatchNorm + ReLU of src formed while staging it (persistent kernel; see ImgConvArgs)
  // persistent kernel with a workspace: queue the partial-slab reduce instead of launching it;
  // flush_wgrad_reduces launches every queued one together (the caller's workspaces must differ)
  int defer_reduce;
};

// launch every deferred weight-gradient reduce (ImgWgradArgs::defer_reduce) as ONE grouped launch on s;
// returns how many there were
int flush_wgrad_reduces(hipStream_t s);
// queued-but-unflushed deferred reduces of this thread, and dropping them (a backward that was
// interrupted between an imgwgrad(defer=True) and its flush leaves them behind)
int pending_wgrad_reduces();
int discard_wgrad_reduces();

bool imgconv_supported(int SH, int SW, int CS, int N, int KH, int KW, int stride, int pad);
// returns whether a.sc_src was added by the launch (false: the caller adds the shortcut gradient)
bool launch_imgconv(const ImgConvArgs& a, hipStream_t s);
// persistent variant (weights resident in LDS, one workgroup per CU streaming images);
// returns false when the shape does not fit it (launch_imgconv then uses the per-image kernel);
// *sc_done: whether the shortcut gradient (a.sc_src) was added
bool launch_imgconv_persistent(const ImgConvArgs& a, hipStream_t s, bool* sc_done = nullptr);
bool imgwgrad_supported(const ImgWgradArgs& a);
// floats of the partial-sum workspace the weight-gradient kernels need (256 workgroup slabs);
// mirrored by ops.wgrad_ws_floats
long imgwgrad_ws_floats(int N, int KC);
void launch_imgwgrad(const ImgWgradArgs& a, hipStream_t s);
// persistent variant (dW accumulated in registers across a workgroup's images);
// returns false when the shape does not fit it
bool launch_imgwgrad_persistent(const ImgWgradArgs& a, hipStream_t s);
// MNIST conv1 (28x28x1, 5x5 SAME, 32 channels, B >= 256): shifted-copy kernels
// (imgconv1_copies.hip); false when the shape is not that layer
bool launch_conv1_copies_fwd(const ImgConvArgs& a, hipStream_t s);
bool launch_conv1_copies_wgrad(const ImgWgradArgs& a, hipStream_t s);


// dw[k] += scale * sum_{p < nblk} ws[p * len + k]   (k >= nw: db[k - nw]), len % 4 == 0.
// Fixed summation order (each thread a strided subset of the partials in order, then the 16
// subsets in order through LDS): bitwise reproducible gradients, no atomics.  One workgroup per
// 64 elements.
void launch_partials_reduce(const float* ws, int nblk, int len, int nw, float* dw, float* db, float scale,
                            hipStream_t s);


// Un-pooling of one 16-B pooled chunk (8 bf16 channels) with its 8 argmax bytes (each 0..3: the
// position in the 2x2 window): out[q] = the chunk with every channel whose argmax != q zeroed.  The
// 2-bit argmax codes give the four byte masks with 2 bit-ops each and v_perm_b32 widens a byte mask
// to the two bytes of its bf16 lane - ~50 VALU for the 4 quadrants against ~160 for the per-word
// xor / compare / select form (rocprof ablation: the un-pooled dY image was a third of the MNIST conv1
// weight-gradient launch).
__device__ __forceinline__ void unpool4(const u32x4_t pv, const u32x2_t am, u32x4_t (&out)[4]) {
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const uint32_t lo = am[h] & 0x01010101u, hi = (am[h] >> 1) & 0x01010101u;
    const uint32_t m[4] = {((lo | hi) ^ 0x01010101u) * 0xFFu, (lo & ~hi) * 0xFFu, (hi & ~lo) * 0xFFu,
                           (lo & hi) * 0xFFu};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      out[q][2 * h] = pv[2 * h] & __builtin_amdgcn_perm(0u, m[q], 0x01010000u);
      out[q][2 * h + 1] = pv[2 * h + 1] & __builtin_amdgcn_perm(0u, m[q], 0x03030202u);
    }
  }
}

}  // namespace dtfe
