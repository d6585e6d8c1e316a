// torch.ops.dtfe.* bindings for the gfx950 kernel library.
//
// Every op writes into caller-provided (pre-allocated) tensors and launches on
// the current HIP stream, so a whole training step built from these ops can be
// captured into a hipGraph (torch.cuda.CUDAGraph) with zero allocations.
#include <ATen/ATen.h>
#include <ATen/hip/HIPContext.h>
#include <torch/library.h>
#include <vector>

#include "../kernels/conv.h"
#include "../kernels/conv_f32.h"
#include "../kernels/imgconv.h"
#include "../kernels/norm.h"
#include "../kernels/elementwise.h"
#include "../kernels/gemm_dense.h"
#include "../kernels/head.h"
#include "../kernels/lstm_seq.h"
#include "../kernels/optim.h"

using at::Tensor;
using c10::optional;

namespace {

hipStream_t cur_stream() { return at::hip::getCurrentHIPStream().stream(); }

template <typename T>
T* ptr_or_null(const optional<Tensor>& t) {
  return (t.has_value() && t->defined()) ? reinterpret_cast<T*>(t->data_ptr()) : nullptr;
}

void check_cuda(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), "dtfe: tensor '", name, "' must be on the GPU (HIP) device");
}

int dtype_code(const Tensor& t) {
  if (t.scalar_type() == at::kBFloat16) return 0;
  if (t.scalar_type() == at::kFloat) return 1;
  TORCH_CHECK(false, "dtfe: unsupported dtype ", t.scalar_type());
}

// ------------------------------------------------------------------- gemm
void gemm(const Tensor& A, int64_t amode, int64_t lda, const Tensor& B, int64_t bmode, int64_t ldb, int64_t M,
          int64_t N, int64_t K, const Tensor& out, int64_t ldc, const optional<Tensor>& bias, int64_t bias_axis,
          int64_t act, double alpha, double beta, bool atomic, int64_t splits, int64_t tile,
          const optional<Tensor>& aux, int64_t ld_aux, int64_t aux_act, int64_t b_ones_row, double keep, int64_t seed,
          const optional<Tensor>& counter, const optional<Tensor>& pooled, const optional<Tensor>& argmax,
          int64_t PH, int64_t PW, int64_t PC, const optional<Tensor>& out2, int64_t ldc2, bool out2_trans,
          const optional<Tensor>& bias_out, const optional<Tensor>& ws, const optional<Tensor>& tile_ctr,
          int64_t a_ones_row, const optional<Tensor>& ones) {
  check_cuda(A, "A");
  check_cuda(B, "B");
  check_cuda(out, "out");
  TORCH_CHECK(A.scalar_type() == B.scalar_type(), "gemm: A and B dtypes differ");
  const int dt = dtype_code(A);
  dtfe::DenseGemmArgs a{};
  a.M = (int)M; a.N = (int)N; a.K = (int)K;
  a.A = A.data_ptr(); a.lda = lda;
  a.B = B.data_ptr(); a.ldb = ldb;
  a.b_ones_row = (int)b_ones_row;
  a.a_ones_row = (int)a_ones_row;
  TORCH_CHECK(a_ones_row < 0 || b_ones_row < 0, "gemm: at most one of a_ones_row / b_ones_row");
  if (splits < 1) splits = 1;
  int bm = 0, bn = 0;
  const int kt = dtfe::gemm_dense_tile_dims((int)tile, bm, bn);
  TORCH_CHECK(kt > 0, "gemm: bad tile id");
  int chunk = (int)((K + splits - 1) / splits);
  chunk = ((chunk + kt - 1) / kt) * kt;
  if (chunk < kt) chunk = kt;
  const int real_splits = (int)((K + chunk - 1) / chunk);
  a.k_chunk = chunk;
  a.out = out.data_ptr(); a.ldc = ldc; a.out_f32 = out.scalar_type() == at::kFloat;
  a.bias = ptr_or_null<float>(bias); a.bias_axis = (int)bias_axis;
  a.act = (int)act; a.alpha = (float)alpha; a.beta = (float)beta; a.atomic = atomic;
  if (real_splits > 1 && !atomic) {
    const int64_t ntiles = ((M + bm - 1) / bm) * ((N + bn - 1) / bn);
    TORCH_CHECK(ws.has_value() && ws->defined() && tile_ctr.has_value() && tile_ctr->defined(),
                "gemm: split-K with a fused epilogue needs ws/tile_ctr");
    TORCH_CHECK(ws->scalar_type() == at::kFloat && ws->numel() >= real_splits * ntiles * bm * bn,
                "gemm: split-K workspace too small");
    TORCH_CHECK(tile_ctr->scalar_type() == at::kInt && tile_ctr->numel() >= ntiles, "gemm: tile counters too small");
    a.ws = ws->data_ptr<float>();
    a.tile_ctr = tile_ctr->data_ptr<int>();
  }
  TORCH_CHECK(!atomic || a.out_f32, "gemm: atomic accumulation needs an fp32 output");
  a.out2 = ptr_or_null<void>(out2); a.ldc2 = ldc2;
  a.out2_f32 = (out2.has_value() && out2->defined()) ? out2->scalar_type() == at::kFloat : 0;
  a.out2_trans = out2_trans;
  a.aux = ptr_or_null<void>(aux); a.ld_aux = ld_aux;
  a.aux_f32 = (aux.has_value() && aux->defined()) ? aux->scalar_type() == at::kFloat : 0;
  a.aux_act = (int)aux_act;
  a.unpool = (pooled.has_value() && pooled->defined()) ? 1 : 0;
  if (a.unpool) {
    TORCH_CHECK(out.scalar_type() == at::kBFloat16, "gemm: unpool epilogue writes bf16");
    a.up.pooled = reinterpret_cast<const dtfe::bf16*>(pooled->data_ptr());
    a.up.argmax = reinterpret_cast<const uint8_t*>(argmax->data_ptr());
    a.up.PH = (int)PH; a.up.PW = (int)PW; a.up.C = (int)PC;
  }
  a.keep = (float)keep; a.seed = (uint64_t)seed; a.counter = ptr_or_null<int64_t>(counter);
  a.bias_out = ptr_or_null<float>(bias_out);
  TORCH_CHECK(!a.bias_out || b_ones_row >= 0 || a_ones_row >= 0, "gemm: bias_out needs a ones row");
  a.ones = ptr_or_null<dtfe::bf16>(ones);
  if (tile == dtfe::GEMM_TILE_SMALL) {
    TORCH_CHECK(real_splits == 1 && dtfe::gemm_small_eligible(dt == 0 ? 0 : 1, a),
                "gemm: the small-tile kernel takes fp32 operands, one split, no un-pool epilogue");
  } else if (tile >= 5) {
    TORCH_CHECK(dtfe::gemm_glds_eligible(dt == 0 ? 0 : 1, (int)amode, (int)bmode, (int)tile, a),
                "gemm: shape / layout not eligible for the global_load_lds tile ", tile);
    // the glds kernels load whole k-tiles of whole operand rows with no bounds checks: every element
    // they may touch must lie inside the tensors
    const int64_t b_rows = b_ones_row >= 0 ? b_ones_row : N;
    const int64_t a_need = amode == 0 ? (M - 1) * lda + K : (K - 1) * lda + M;
    const int64_t b_need = bmode == 0 ? (b_rows - 1) * ldb + K : (K - 1) * ldb + b_rows;
    TORCH_CHECK(A.numel() >= a_need && B.numel() >= b_need, "gemm: operands smaller than M/N/K/ld imply");
  }
  dtfe::launch_gemm_dense(dt == 0 ? 0 : 1, (int)amode, (int)bmode, (int)tile, real_splits, a, cur_stream());
}

// gemm_group(anchor, begin): begin / end a grouped launch on the current stream (gemm_dense.h);
// `anchor` is any tensor on the launch device (dispatch only)
void gemm_group(const Tensor& anchor, bool begin) {
  check_cuda(anchor, "anchor");
  if (begin) dtfe::glds_group_begin();
  else dtfe::glds_group_end(cur_stream());
}

// ------------------------------------------------------------------- conv
dtfe::ConvGeom geom(int64_t B, int64_t H, int64_t W, int64_t C, int64_t Cout, int64_t OH, int64_t OW, int64_t KH,
                    int64_t KW, int64_t stride, int64_t pad, int64_t pool) {
  dtfe::ConvGeom g;
  g.B = (int)B; g.H = (int)H; g.W = (int)W; g.C = (int)C; g.Cout = (int)Cout; g.OH = (int)OH; g.OW = (int)OW;
  g.KH = (int)KH; g.KW = (int)KW; g.stride = (int)stride; g.pad = (int)pad; g.pool_order = (int)pool;
  return g;
}

void conv_fwd(const Tensor& x, const Tensor& w, const optional<Tensor>& bias, const Tensor& y,
              const optional<Tensor>& argmax, int64_t B, int64_t H, int64_t W, int64_t C, int64_t Cout, int64_t OH,
              int64_t OW, int64_t KH, int64_t KW, int64_t stride, int64_t pad, bool pool, int64_t act,
              const optional<Tensor>& bn_stats) {
  check_cuda(x, "x");
  if (x.scalar_type() == at::kFloat) {  // exact-fp32 path (--dtype fp32): conv_f32.hip
    TORCH_CHECK(w.scalar_type() == at::kFloat && y.scalar_type() == at::kFloat && !(bn_stats.has_value() && bn_stats->defined()),
                "conv_fwd (fp32): fp32 x / w / y, no BatchNorm statistics");
    TORCH_CHECK(!pool || ((OH | OW) & 1) == 0, "conv_fwd (fp32): pool needs even output dims");
    dtfe::ConvF32Args f{};
    f.g = geom(B, H, W, C, Cout, OH, OW, KH, KW, stride, pad, pool);
    f.src = x.data_ptr<float>(); f.w = w.data_ptr<float>(); f.bias = ptr_or_null<float>(bias);
    f.out = y.data_ptr<float>(); f.argmax = ptr_or_null<uint8_t>(argmax); f.act = (int)act;
    TORCH_CHECK(y.numel() == B * OH * OW * Cout / (pool ? 4 : 1) && x.numel() == B * H * W * C &&
                w.numel() == Cout * KH * KW * C, "conv_fwd (fp32): shapes");
    dtfe::launch_conv_fwd_f32(f, cur_stream());
    return;
  }
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && w.scalar_type() == at::kBFloat16, "conv_fwd: bf16 or fp32");
  dtfe::ConvFwdArgs a{};
  if (bn_stats.has_value() && bn_stats->defined()) {
    TORCH_CHECK(bn_stats->scalar_type() == at::kFloat && bn_stats->is_contiguous() && bn_stats->numel() >= 2 * Cout,
                "conv_fwd: bn_stats must be f32 [2][Cout]");
    a.bn_stats = bn_stats->data_ptr<float>();
  }
  a.g = geom(B, H, W, C, Cout, OH, OW, KH, KW, stride, pad, pool);
  a.x = reinterpret_cast<const dtfe::bf16*>(x.data_ptr());
  a.w = reinterpret_cast<const dtfe::bf16*>(w.data_ptr());
  a.bias = ptr_or_null<float>(bias);
  a.y = reinterpret_cast<dtfe::bf16*>(y.data_ptr());
  a.argmax = ptr_or_null<uint8_t>(argmax);
  a.act = (int)act;
  dtfe::launch_conv_fwd(a, cur_stream());
}

void conv_dgrad(const Tensor& dy, const Tensor& wt, const Tensor& dx, int64_t B, int64_t H, int64_t W, int64_t C,
                int64_t Cout, int64_t OH, int64_t OW, int64_t KH, int64_t KW, int64_t stride, int64_t pad,
                const optional<Tensor>& pooled, const optional<Tensor>& argmax, const optional<Tensor>& relu_mask,
                bool accumulate, const optional<Tensor>& bnb_x, const optional<Tensor>& bnb_y,
                const optional<Tensor>& bnb_mean, const optional<Tensor>& bnb_invstd, const optional<Tensor>& bnb_gamma,
                const optional<Tensor>& bnb_beta, const optional<Tensor>& bnb_stats, int64_t bnb_act,
                const optional<Tensor>& acc_src, const optional<Tensor>& acc_mask) {
  check_cuda(dy, "dy");
  if (dy.scalar_type() == at::kFloat) {  // exact-fp32 path (--dtype fp32): conv_f32.hip
    TORCH_CHECK(wt.scalar_type() == at::kFloat && dx.scalar_type() == at::kFloat && stride == 1 && !accumulate &&
                    !(pooled.has_value() && pooled->defined()) && !(bnb_stats.has_value() && bnb_stats->defined()),
                "conv_dgrad (fp32): fp32 tensors, stride 1, optional ReLU mask only");
    TORCH_CHECK(dx.numel() == B * H * W * C && dy.numel() == B * OH * OW * Cout && wt.numel() == C * KH * KW * Cout,
                "conv_dgrad (fp32): shapes");
    dtfe::ConvF32Args f{};
    f.g = geom(B, H, W, C, Cout, OH, OW, KH, KW, stride, pad, 0);
    f.src = dy.data_ptr<float>(); f.w = wt.data_ptr<float>(); f.out = dx.data_ptr<float>();
    if (relu_mask.has_value() && relu_mask->defined()) {
      TORCH_CHECK(relu_mask->scalar_type() == at::kFloat && relu_mask->numel() == dx.numel(), "conv_dgrad (fp32): mask");
      f.relu_mask = relu_mask->data_ptr<float>();
    }
    dtfe::launch_conv_dgrad_f32(f, cur_stream());
    return;
  }
  dtfe::ConvDgradArgs a{};
  a.accumulate = accumulate ? 1 : 0;
  if (bnb_stats.has_value() && bnb_stats->defined()) {
    TORCH_CHECK(bnb_x.has_value() && bnb_x->defined() && bnb_mean.has_value() && bnb_invstd.has_value() &&
                    bnb_gamma.has_value(), "conv_dgrad: BN-backward statistics need x, mean, invstd, gamma");
    TORCH_CHECK(bnb_x->numel() == dx.numel() && bnb_x->scalar_type() == at::kBFloat16, "conv_dgrad: bnb_x shape/dtype");
    TORCH_CHECK(bnb_stats->numel() >= 2 * C && bnb_stats->scalar_type() == at::kFloat, "conv_dgrad: bnb_stats [2][C] fp32");
    TORCH_CHECK(bnb_mean->numel() >= C && bnb_invstd->numel() >= C && bnb_gamma->numel() >= C, "conv_dgrad: BN params");
    const bool bits = bnb_y.has_value() && bnb_y->defined() && bnb_y->scalar_type() == at::kByte;
    if (bnb_y.has_value() && bnb_y->defined())
      TORCH_CHECK(bits ? bnb_y->numel() == dx.numel() / 8 : (bnb_y->numel() == dx.numel() && bnb_y->scalar_type() == at::kBFloat16),
                  "conv_dgrad: bnb_y shape/dtype (bf16 output, or its uint8 [R][C/8] ReLU bit mask)");
    if (bnb_beta.has_value() && bnb_beta->defined()) TORCH_CHECK(bnb_beta->numel() >= C, "conv_dgrad: bnb_beta");
    a.bnb_x = reinterpret_cast<const dtfe::bf16*>(bnb_x->data_ptr());
    if (bits) a.bnb_ymask = bnb_y->data_ptr<uint8_t>();
    else a.bnb_y = ptr_or_null<dtfe::bf16>(bnb_y);
    a.bnb_mean = bnb_mean->data_ptr<float>();
    a.bnb_invstd = bnb_invstd->data_ptr<float>();
    a.bnb_gamma = bnb_gamma->data_ptr<float>();
    a.bnb_beta = ptr_or_null<float>(bnb_beta);
    a.bnb_stats = bnb_stats->data_ptr<float>();
    a.bnb_act = (int)bnb_act;
  }
  if (acc_src.has_value() && acc_src->defined()) {
    TORCH_CHECK(accumulate && acc_src->numel() == dx.numel() && acc_src->scalar_type() == at::kBFloat16 &&
                    acc_mask.has_value() && acc_mask->defined() && acc_mask->scalar_type() == at::kByte &&
                    acc_mask->numel() == dx.numel() / 8,
                "conv_dgrad: acc_src (bf16, dx's shape) needs accumulate and its uint8 [R][C/8] bit mask");
    a.acc_src = reinterpret_cast<const dtfe::bf16*>(acc_src->data_ptr());
    a.acc_mask = acc_mask->data_ptr<uint8_t>();
  }
  a.g = geom(B, H, W, C, Cout, OH, OW, KH, KW, stride, pad, 0);
  a.dy = reinterpret_cast<const dtfe::bf16*>(dy.data_ptr());
  a.wt = reinterpret_cast<const dtfe::bf16*>(wt.data_ptr());
  a.dx = reinterpret_cast<dtfe::bf16*>(dx.data_ptr());
  a.relu_mask = ptr_or_null<dtfe::bf16>(relu_mask);
  a.unpool = (pooled.has_value() && pooled->defined()) ? 1 : 0;
  if (a.unpool) {
    a.up.pooled = reinterpret_cast<const dtfe::bf16*>(pooled->data_ptr());
    a.up.argmax = reinterpret_cast<const uint8_t*>(argmax->data_ptr());
    a.up.PH = (int)H; a.up.PW = (int)W; a.up.C = (int)C;
  }
  dtfe::launch_conv_dgrad(a, cur_stream());
}

// [stats, gamma, beta, mean, invstd, moving_mean, moving_var] of a BatchNorm + ReLU formed on a
// whole-image conv's source (the last four may be undefined: nothing saved / updated)
dtfe::BnSrc bn_src_of(const optional<at::TensorList>& t, long R, int64_t C, double eps, double momentum, bool save) {
  dtfe::BnSrc b{};
  if (!t.has_value() || t->empty()) return b;
  TORCH_CHECK(t->size() == 7, "bn_src: [stats, gamma, beta, mean, invstd, moving_mean, moving_var]");
  const auto& v = *t;
  for (int i = 0; i < 3; ++i) {
    check_cuda(v[i], "bn_src");
    TORCH_CHECK(v[i].scalar_type() == at::kFloat && v[i].numel() >= (i == 0 ? 2 : 1) * C, "bn_src: fp32 [C] / [2][C]");
  }
  b.stats = v[0].data_ptr<float>();
  b.gamma = v[1].data_ptr<float>();
  b.beta = v[2].data_ptr<float>();
  auto opt = [&](int i) { return save && v[i].defined() ? v[i].data_ptr<float>() : nullptr; };
  b.mean = opt(3); b.invstd = opt(4); b.moving_mean = opt(5); b.moving_var = opt(6);
  TORCH_CHECK((b.moving_mean == nullptr) == (b.moving_var == nullptr), "bn_src: both moving averages or neither");
  b.R = R; b.eps = (float)eps; b.momentum = (float)momentum;
  return b;
}

bool imgconv(const optional<Tensor>& src, const optional<Tensor>& src_pooled, const optional<Tensor>& src_argmax,
             const Tensor& w, const optional<Tensor>& bias, const Tensor& y, const optional<Tensor>& argmax,
             const optional<Tensor>& relu_mask, int64_t B, int64_t SH, int64_t SW, int64_t CS, int64_t OH, int64_t OW,
             int64_t N, int64_t KH, int64_t KW, int64_t stride, int64_t pad, bool flip_taps, int64_t act, bool pool,
             int64_t dil, const optional<Tensor>& sc_src, int64_t sc_stride, const optional<Tensor>& tstamp,
             const optional<at::TensorList>& bn_src, double bn_eps, double bn_momentum, bool bn_save) {
  check_cuda(w, "w");
  TORCH_CHECK((src.has_value() && src->defined()) != (src_pooled.has_value() && src_pooled->defined()),
              "imgconv: exactly one of src / src_pooled");
  dtfe::ImgConvArgs a{};
  a.B = (int)B; a.SH = (int)SH; a.SW = (int)SW; a.CS = (int)CS; a.OH = (int)OH; a.OW = (int)OW; a.N = (int)N;
  a.KH = (int)KH; a.KW = (int)KW; a.stride = (int)stride; a.pad = (int)pad; a.flip_taps = flip_taps;
  a.dil = (int)dil;
  a.src = ptr_or_null<dtfe::bf16>(src);
  a.src_pooled = ptr_or_null<dtfe::bf16>(src_pooled);
  a.src_argmax = ptr_or_null<uint8_t>(src_argmax);
  TORCH_CHECK(a.src || a.src_argmax, "imgconv: src_pooled needs src_argmax");
  a.w = reinterpret_cast<const dtfe::bf16*>(w.data_ptr());
  a.bias = ptr_or_null<float>(bias);
  a.act = (int)act; a.pool = pool;
  a.y = reinterpret_cast<dtfe::bf16*>(y.data_ptr());
  a.argmax = ptr_or_null<uint8_t>(argmax);
  a.relu_mask = ptr_or_null<dtfe::bf16>(relu_mask);
  TORCH_CHECK(w.numel() == N * KH * KW * CS, "imgconv: weight size");
  TORCH_CHECK(y.numel() == B * OH * OW * N / (pool ? 4 : 1), "imgconv: output size");
  a.tstamp = tstamp.has_value() && tstamp->defined() ? reinterpret_cast<uint64_t*>(tstamp->data_ptr()) : nullptr;
  a.bns = bn_src_of(bn_src, (long)B * SH * SW, CS, bn_eps, bn_momentum, bn_save);
  TORCH_CHECK(!a.bns.stats || a.src, "imgconv: BN-on-load needs a plain source");
  a.sc_src = ptr_or_null<dtfe::bf16>(sc_src);
  if (a.sc_src) {
    TORCH_CHECK(sc_stride >= 1 && OH % sc_stride == 0 && OW % sc_stride == 0 && sc_src->dim() == 4 &&
                    sc_src->size(0) == B && sc_src->size(1) == OH / sc_stride && sc_src->size(2) == OW / sc_stride &&
                    sc_src->size(3) >= N,
                "imgconv: shortcut gradient [B][OH/s][OW/s][>= N]");
    a.sc_stride = (int)sc_stride;
    a.sc_C = (int)sc_src->size(3);
  }
  return dtfe::launch_imgconv(a, cur_stream());
}

// MNIST conv1 forward with the step's batch sampling fused in (imgconv1_copies.hip): samples B rows
// of the uint8 dataset, writes the bf16 images to x (the weight gradient's input) and the labels,
// clears the accumulators in `zero`, and runs conv1 + bias + ReLU + 2x2 max-pool(+argmax).
void conv1_gather_fwd(const Tensor& images, const Tensor& labels_src, int64_t seed, const Tensor& counter,
                      const Tensor& done, const Tensor& labels_dst, const Tensor& x, const Tensor& w,
                      const optional<Tensor>& bias, const Tensor& y, const Tensor& argmax, at::TensorList zero) {
  check_cuda(images, "images");
  TORCH_CHECK(images.scalar_type() == at::kByte && images.dim() == 2 && images.size(1) == 784,
              "conv1_gather_fwd: uint8 [rows][784] dataset");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && x.numel() % 784 == 0, "conv1_gather_fwd: bf16 x [B][28][28]");
  dtfe::ImgConvArgs a{};
  a.B = (int)(x.numel() / 784); a.SH = a.SW = 28; a.CS = 1; a.OH = a.OW = 28; a.N = 32;
  a.KH = a.KW = 5; a.stride = 1; a.pad = 2; a.dil = 1;
  a.src = reinterpret_cast<const dtfe::bf16*>(x.data_ptr());
  a.w = reinterpret_cast<const dtfe::bf16*>(w.data_ptr());
  a.bias = ptr_or_null<float>(bias);
  a.act = dtfe::ACT_RELU; a.pool = 1;
  a.y = reinterpret_cast<dtfe::bf16*>(y.data_ptr());
  a.argmax = reinterpret_cast<uint8_t*>(argmax.data_ptr());
  TORCH_CHECK(w.numel() == 32 * 25 && y.numel() == (int64_t)a.B * 14 * 14 * 32 && argmax.numel() == y.numel(),
              "conv1_gather_fwd: MNIST conv1 shapes");
  a.g_src = images.data_ptr<uint8_t>(); a.g_rows = images.size(0); a.g_seed = (uint64_t)seed;
  // an empty `done` leaves the counter alone (the caller advances it later in the step)
  a.g_counter = counter.data_ptr<int64_t>();
  a.g_done = done.numel() ? reinterpret_cast<uint32_t*>(done.data_ptr()) : nullptr;
  a.g_labels_src = labels_src.data_ptr<int32_t>(); a.g_labels_dst = labels_dst.data_ptr<int32_t>();
  TORCH_CHECK(zero.size() <= 4, "conv1_gather_fwd: at most 4 zero ranges");
  for (const Tensor& z : zero) {
    TORCH_CHECK(z.is_contiguous() && (z.numel() * z.element_size()) % 4 == 0, "conv1_gather_fwd: zero ranges");
    a.zptr[a.nz] = reinterpret_cast<uint32_t*>(z.data_ptr());
    a.zlen[a.nz++] = (long)(z.numel() * z.element_size() / 4);
  }
  TORCH_CHECK(dtfe::launch_conv1_copies_fwd(a, cur_stream()), "conv1_gather_fwd: needs B >= 256");
}

void imgwgrad(const Tensor& src, const optional<Tensor>& dy, const optional<Tensor>& dy_pooled,
              const optional<Tensor>& dy_argmax, const Tensor& dw, const optional<Tensor>& db, int64_t B, int64_t SH,
              int64_t SW, int64_t CS, int64_t OH, int64_t OW, int64_t N, int64_t KH, int64_t KW, int64_t stride,
              int64_t pad, double scale, const optional<Tensor>& ws, int64_t max_blocks,
              const optional<at::TensorList>& bn_src, double bn_eps, bool defer) {
  check_cuda(src, "src");
  dtfe::ImgWgradArgs a{};
  a.defer_reduce = defer ? 1 : 0;
  a.bns = bn_src_of(bn_src, (long)B * SH * SW, CS, bn_eps, 0.0, false);
  a.max_blocks = (int)max_blocks;
  if (ws.has_value() && ws->defined()) {
    TORCH_CHECK(ws->scalar_type() == at::kFloat && ws->numel() >= dtfe::imgwgrad_ws_floats((int)N, (int)(KH * KW * CS)),
                "imgwgrad: workspace too small (ops.wgrad_ws_floats)");
    a.ws = ws->data_ptr<float>();
  }
  a.B = (int)B; a.SH = (int)SH; a.SW = (int)SW; a.CS = (int)CS; a.OH = (int)OH; a.OW = (int)OW; a.N = (int)N;
  a.KH = (int)KH; a.KW = (int)KW; a.stride = (int)stride; a.pad = (int)pad;
  a.src = reinterpret_cast<const dtfe::bf16*>(src.data_ptr());
  a.dy = ptr_or_null<dtfe::bf16>(dy);
  a.dy_pooled = ptr_or_null<dtfe::bf16>(dy_pooled);
  a.dy_argmax = ptr_or_null<uint8_t>(dy_argmax);
  TORCH_CHECK((a.dy != nullptr) != (a.dy_pooled != nullptr), "imgwgrad: exactly one of dy / dy_pooled");
  TORCH_CHECK(dw.scalar_type() == at::kFloat && dw.numel() == N * KH * KW * CS, "imgwgrad: dw");
  a.dw = dw.data_ptr<float>();
  a.db = ptr_or_null<float>(db);
  a.scale = (float)scale;
  dtfe::launch_imgwgrad(a, cur_stream());
}

void conv_wgrad(const Tensor& dz, const Tensor& x, const Tensor& dw, const optional<Tensor>& db, int64_t B, int64_t H,
                int64_t W, int64_t C, int64_t Cout, int64_t OH, int64_t OW, int64_t KH, int64_t KW, int64_t stride,
                int64_t pad, double scale) {
  check_cuda(dz, "dz");
  TORCH_CHECK(dw.scalar_type() == at::kFloat, "conv_wgrad: fp32 grad buffer");
  if (dz.scalar_type() == at::kFloat) {  // exact-fp32 path (--dtype fp32): conv_f32.hip
    TORCH_CHECK(x.scalar_type() == at::kFloat && dz.numel() == B * OH * OW * Cout && x.numel() == B * H * W * C &&
                    dw.numel() == Cout * KH * KW * C, "conv_wgrad (fp32): fp32 dz / x, shapes");
    dtfe::ConvF32Args f{};
    f.g = geom(B, H, W, C, Cout, OH, OW, KH, KW, stride, pad, 0);
    f.src = dz.data_ptr<float>(); f.x = x.data_ptr<float>(); f.dw = dw.data_ptr<float>();
    f.db = ptr_or_null<float>(db); f.scale = (float)scale;
    dtfe::launch_conv_wgrad_f32(f, cur_stream());
    return;
  }
  dtfe::ConvWgradArgs a{};
  a.g = geom(B, H, W, C, Cout, OH, OW, KH, KW, stride, pad, 0);
  a.dz = reinterpret_cast<const dtfe::bf16*>(dz.data_ptr());
  a.x = reinterpret_cast<const dtfe::bf16*>(x.data_ptr());
  a.dw = dw.data_ptr<float>();
  a.db = ptr_or_null<float>(db);
  a.scale = (float)scale;
  dtfe::launch_conv_wgrad(a, cur_stream());
}

// 2x2 un-pool of a pooled fp32 gradient (argmax routing) and the [O][T][C] -> [C][T][O] weight
// transpose: the two data movers of the fp32 CNN step (conv_f32.hip)
void unpool_f32(const Tensor& g, const Tensor& argmax, const Tensor& out, int64_t B, int64_t PH, int64_t PW,
                int64_t C) {
  check_cuda(g, "g");
  TORCH_CHECK(g.scalar_type() == at::kFloat && out.scalar_type() == at::kFloat && argmax.scalar_type() == at::kByte &&
                  g.numel() == B * PH * PW * C && argmax.numel() == g.numel() && out.numel() == 4 * g.numel(),
              "unpool_f32: fp32 g [B][PH][PW][C], uint8 argmax, fp32 out [B][2PH][2PW][C]");
  dtfe::launch_unpool_f32(g.data_ptr<float>(), argmax.data_ptr<uint8_t>(), out.data_ptr<float>(), (int)B, (int)PH,
                          (int)PW, (int)C, cur_stream());
}

// MNIST conv1 weight gradient at fp32 from the pooled gradient (conv_f32.hip); false: shape not covered
bool conv1_wgrad_pooled_f32(const Tensor& dp, const Tensor& argmax, const Tensor& x, const Tensor& dw,
                            const optional<Tensor>& db, const Tensor& ws, int64_t B, int64_t H, int64_t W, int64_t K,
                            double scale) {
  check_cuda(dp, "dp");
  TORCH_CHECK(dp.scalar_type() == at::kFloat && x.scalar_type() == at::kFloat && dw.scalar_type() == at::kFloat &&
                  argmax.scalar_type() == at::kByte && ws.scalar_type() == at::kFloat,
              "conv1_wgrad_pooled_f32: fp32 dp / x / dw / ws, uint8 argmax");
  TORCH_CHECK(dp.is_contiguous() && argmax.is_contiguous() && x.is_contiguous() && dp.numel() == B * (H / 2) * (W / 2) * 32 &&
                  argmax.numel() == dp.numel() && x.numel() == B * H * W && dw.numel() == 32 * K * K &&
                  (!db.has_value() || !db->defined() || db->numel() == 32),
              "conv1_wgrad_pooled_f32: dp [B][H/2][W/2][32], x [B][H][W][1], dw [32][K][K][1], db [32]");
  const dtfe::ConvGeom g = geom(B, H, W, 1, 32, H, W, K, K, 1, K / 2, 0);
  return dtfe::launch_conv1_wgrad_pooled_f32(dp.data_ptr<float>(), argmax.data_ptr<uint8_t>(), x.data_ptr<float>(),
                                             dw.data_ptr<float>(), ptr_or_null<float>(db), ws.data_ptr<float>(),
                                             ws.numel(), g, (float)scale, cur_stream());
}

void transpose_taps_f32(const Tensor& in, const Tensor& out, int64_t O, int64_t T, int64_t C) {
  check_cuda(in, "in");
  TORCH_CHECK(in.scalar_type() == at::kFloat && out.scalar_type() == at::kFloat && in.numel() == O * T * C &&
                  out.numel() == in.numel() && in.is_contiguous() && out.is_contiguous(), "transpose_taps_f32: shapes");
  dtfe::launch_transpose_taps_f32(in.data_ptr<float>(), out.data_ptr<float>(), (int)O, (int)T, (int)C, cur_stream());
}

// ------------------------------------------------------------------- head
// fp32 fused head (head.hip head_xent_f32_kernel); false: shape not instantiated (caller: GEMMs + softmax_xent)
bool head_xent_f32(const Tensor& h, const Tensor& w, const optional<Tensor>& b, const Tensor& labels, const Tensor& dz,
                   const Tensor& dl, const Tensor& loss_sum, const Tensor& correct, const optional<Tensor>& logits,
                   double scale, double inv_keep, const optional<Tensor>& step_counter) {
  check_cuda(h, "h");
  TORCH_CHECK(h.scalar_type() == at::kFloat && w.scalar_type() == at::kFloat && dz.scalar_type() == at::kFloat &&
                  dl.scalar_type() == at::kFloat && labels.scalar_type() == at::kInt && h.dim() == 2 && w.dim() == 2 &&
                  h.is_contiguous() && w.is_contiguous() && dz.is_contiguous() && dl.is_contiguous(),
              "head_xent_f32: fp32 h [B][K], W [NC][K], dz, dl; int32 labels");
  dtfe::HeadF32Args a{};
  a.B = (int)h.size(0); a.K = (int)h.size(1); a.NC = (int)w.size(0);
  TORCH_CHECK(w.size(1) == a.K && dz.numel() == h.numel() && dl.numel() == (int64_t)a.B * a.NC && labels.numel() >= a.B,
              "head_xent_f32: shapes");
  a.h = h.data_ptr<float>(); a.w = w.data_ptr<float>(); a.b = ptr_or_null<float>(b);
  a.labels = labels.data_ptr<int32_t>();
  a.scale = (float)scale; a.inv_keep = (float)inv_keep;
  a.dz = dz.data_ptr<float>(); a.dl = dl.data_ptr<float>();
  a.logits_out = ptr_or_null<float>(logits);
  TORCH_CHECK(!a.logits_out || logits->numel() == dl.numel(), "head_xent_f32: logits [B][NC]");
  a.loss_sum = loss_sum.data_ptr<float>(); a.correct = correct.data_ptr<int32_t>();
  a.step_counter = nullptr;
  if (step_counter.has_value() && step_counter->defined()) {
    TORCH_CHECK(step_counter->scalar_type() == at::kLong && step_counter->is_cuda(), "head_xent_f32: int64 step_counter");
    a.step_counter = step_counter->data_ptr<int64_t>();
  }
  return dtfe::launch_head_xent_f32(a, cur_stream());
}

void head_xent(const Tensor& h, const Tensor& w, const optional<Tensor>& b, const Tensor& labels, const Tensor& dz,
               const Tensor& dl, const optional<Tensor>& loss_sum, const optional<Tensor>& correct,
               const optional<Tensor>& logits, double scale, double inv_keep, const optional<Tensor>& step_counter,
               const optional<Tensor>& parts) {
  check_cuda(h, "h");
  TORCH_CHECK(dl.scalar_type() == at::kBFloat16 && dl.dim() == 2, "head_xent: dl must be bf16 [B][ld]");
  dtfe::HeadArgs a{};
  a.B = (int)h.size(0); a.K = (int)h.size(1); a.NC = (int)(w.numel() / a.K);
  TORCH_CHECK(dl.size(1) >= a.NC && dl.size(1) <= 64, "head_xent: dl row must hold NC classes");
  a.h = reinterpret_cast<const dtfe::bf16*>(h.data_ptr());
  a.w = reinterpret_cast<const dtfe::bf16*>(w.data_ptr());
  a.b = ptr_or_null<float>(b);
  a.labels = labels.data_ptr<int32_t>();
  a.scale = (float)scale; a.inv_keep = (float)inv_keep;
  a.dz = reinterpret_cast<dtfe::bf16*>(dz.data_ptr());
  a.dl = reinterpret_cast<dtfe::bf16*>(dl.data_ptr()); a.ld_dl = (int)dl.size(1);
  a.loss_sum = ptr_or_null<float>(loss_sum); a.correct = ptr_or_null<int32_t>(correct);
  a.logits_out = ptr_or_null<float>(logits);
  if (step_counter.has_value() && step_counter->defined()) {
    TORCH_CHECK(step_counter->scalar_type() == at::kLong && step_counter->is_cuda(), "head_xent: int64 step_counter");
    a.step_counter = step_counter->data_ptr<int64_t>();
  }
  if (parts.has_value() && parts->defined()) {
    TORCH_CHECK(parts->scalar_type() == at::kFloat && parts->is_cuda() && parts->numel() >= 2 * ((a.B + 3) / 4),
                "head_xent: parts must be fp32 [>= 2 * ceil(B / 4)]");
    a.parts = parts->data_ptr<float>();
  }
  dtfe::launch_head_xent(a, cur_stream());
}

void head_wgrad(const Tensor& dl, const Tensor& h, const Tensor& dw, const optional<Tensor>& db, int64_t nc,
                double scale, const optional<Tensor>& parts, const optional<Tensor>& loss_sum,
                const optional<Tensor>& correct) {
  check_cuda(h, "h");
  TORCH_CHECK(dl.scalar_type() == at::kBFloat16 && h.scalar_type() == at::kBFloat16 && dl.dim() == 2 && h.dim() == 2,
              "head_wgrad: bf16 dl [B][ld] and h [B][K]");
  TORCH_CHECK(dw.scalar_type() == at::kFloat && dw.dim() == 2 && dw.size(0) == nc && dw.stride(1) == 1,
              "head_wgrad: fp32 dw [NC][>=K]");
  TORCH_CHECK(dl.size(0) == h.size(0) && dl.stride(1) == 1 && h.stride(1) == 1 && dl.size(1) >= nc,
              "head_wgrad: batch / layout mismatch");
  dtfe::HeadWgradArgs a{};
  a.B = (int)h.size(0); a.K = (int)h.size(1); a.NC = (int)nc;
  TORCH_CHECK(dw.size(1) >= a.K, "head_wgrad: dw rows shorter than K");
  a.dl = reinterpret_cast<const dtfe::bf16*>(dl.data_ptr()); a.ld_dl = (int)dl.stride(0);
  a.h = reinterpret_cast<const dtfe::bf16*>(h.data_ptr()); a.ldh = (int)h.stride(0);
  a.dw = dw.data_ptr<float>(); a.ldw = (int)dw.stride(0);
  if (db.has_value() && db->defined()) {
    TORCH_CHECK(db->scalar_type() == at::kFloat && db->numel() >= nc, "head_wgrad: fp32 db [NC]");
    a.db = db->data_ptr<float>();
  }
  a.scale = (float)scale;
  if (parts.has_value() && parts->defined()) {
    TORCH_CHECK(parts->scalar_type() == at::kFloat && parts->is_cuda() && parts->numel() >= 2 * ((a.B + 3) / 4),
                "head_wgrad: parts must be fp32 [>= 2 * ceil(B / 4)] (head_xent's)");
    TORCH_CHECK(loss_sum.has_value() && loss_sum->scalar_type() == at::kFloat && correct.has_value() &&
                correct->scalar_type() == at::kInt, "head_wgrad: parts need fp32 loss_sum and int32 correct");
    a.parts = parts->data_ptr<float>(); a.nparts = (a.B + 3) / 4;
    a.loss_sum = loss_sum->data_ptr<float>(); a.correct = correct->data_ptr<int32_t>();
  }
  dtfe::launch_head_wgrad(a, cur_stream());
}

// -------------------------------------------------------------- optimizer
// segs: int64 [nseg, 6] = (off, R, T, C, w16_ptr, wt16_ptr)
// work: int64 [nwork, 7] = (kind, seg, t, r0, c0, start, count)
// returns a device blob holding both struct arrays
Tensor opt_pack(const Tensor& segs, const Tensor& work, const Tensor& device_like) {
  TORCH_CHECK(segs.device().is_cpu() && work.device().is_cpu(), "opt_pack: CPU int64 tables");
  auto S = segs.contiguous(), Wk = work.contiguous();
  const int64_t ns = S.size(0), nw = Wk.size(0);
  std::vector<dtfe::OptSeg> vs(ns);
  std::vector<dtfe::OptWork> vw(nw);
  const int64_t* s = S.data_ptr<int64_t>();
  const int64_t* w = Wk.data_ptr<int64_t>();
  for (int64_t i = 0; i < ns; ++i) {
    vs[i].off = s[i * 6 + 0];
    vs[i].R = (int)s[i * 6 + 1]; vs[i].T = (int)s[i * 6 + 2]; vs[i].C = (int)s[i * 6 + 3];
    vs[i].w16 = reinterpret_cast<dtfe::bf16*>(s[i * 6 + 4]);
    vs[i].wt16 = reinterpret_cast<dtfe::bf16*>(s[i * 6 + 5]);
  }
  for (int64_t i = 0; i < nw; ++i) {
    vw[i].kind = (int)w[i * 7 + 0]; vw[i].seg = (int)w[i * 7 + 1]; vw[i].t = (int)w[i * 7 + 2];
    vw[i].r0 = (int)w[i * 7 + 3]; vw[i].c0 = (int)w[i * 7 + 4];
    vw[i].start = w[i * 7 + 5]; vw[i].count = w[i * 7 + 6];
  }
  const size_t bs = ns * sizeof(dtfe::OptSeg), bw = nw * sizeof(dtfe::OptWork);
  const size_t off_w = (bs + 255) / 256 * 256;
  Tensor host = at::empty({(int64_t)(off_w + bw)}, at::TensorOptions().dtype(at::kByte));
  std::memcpy(host.data_ptr(), vs.data(), bs);
  std::memcpy((char*)host.data_ptr() + off_w, vw.data(), bw);
  return host.to(device_like.device());
}

// apply_wait_next(done, seen, segs): the NEXT apply_gradients call's items of the segments in the bit mask
// `segs` wait on the device-side counter pair (OptArgs::wait_done / wait_seen) - a gradient produced on
// another stream with no graph edge to the optimizer launch (the CNN's conv2 weight-gradient branch)
struct ApplyWait { int* done = nullptr; int* seen = nullptr; uint32_t segs = 0; };
thread_local ApplyWait g_apply_wait;
void apply_wait_next(const Tensor& done, const Tensor& seen, int64_t segs) {
  check_cuda(done, "done");
  TORCH_CHECK(done.scalar_type() == at::kInt && seen.scalar_type() == at::kInt && done.numel() >= 1 && seen.numel() >= 1,
              "apply_wait_next: int32 counters");
  g_apply_wait = ApplyWait{done.data_ptr<int>(), seen.data_ptr<int>(), (uint32_t)segs};
}
void epoch_signal(const Tensor& ctr) {
  check_cuda(ctr, "ctr");
  TORCH_CHECK(ctr.scalar_type() == at::kInt && ctr.numel() >= 1, "epoch_signal: int32 counter");
  dtfe::launch_epoch_signal(ctr.data_ptr<int>(), cur_stream());
}

void apply_gradients(int64_t kind, const Tensor& p, const optional<Tensor>& g, const optional<Tensor>& g16,
                     double gscale, const optional<Tensor>& s1, const optional<Tensor>& s2, double lr, double beta1,
                     double beta2, double eps, double momentum, double rho, const optional<Tensor>& beta_pow,
                     const optional<Tensor>& global_step, int64_t gs_inc, const Tensor& done, const Tensor& blob,
                     int64_t nseg, int64_t nwork, int64_t group) {
  check_cuda(p, "p");
  // group: 0 = launch now; 1 = queue these args; 2 = queue and launch every queued optimizer in
  // ONE grouped launch (same kind, disjoint var lists: e.g. the GAN's two Adams)
  thread_local std::vector<dtfe::OptArgs> pending;
  dtfe::OptArgs a{};
  a.kind = (int)kind;
  a.p = p.data_ptr<float>();
  a.g = ptr_or_null<float>(g);
  a.g16 = ptr_or_null<dtfe::bf16>(g16);
  TORCH_CHECK((a.g != nullptr) != (a.g16 != nullptr), "apply_gradients: exactly one of g / g16");
  a.gscale = (float)gscale;
  a.s1 = ptr_or_null<float>(s1); a.s2 = ptr_or_null<float>(s2);
  a.lr = (float)lr; a.beta1 = (float)beta1; a.beta2 = (float)beta2; a.eps = (float)eps;
  a.momentum = (float)momentum; a.rho = (float)rho;
  a.beta_pow = ptr_or_null<float>(beta_pow);
  a.global_step = ptr_or_null<int32_t>(global_step);
  a.gs_inc = (int)gs_inc;
  a.done_counter = reinterpret_cast<uint32_t*>(done.data_ptr());
  const size_t bs = nseg * sizeof(dtfe::OptSeg);
  const size_t off_w = (bs + 255) / 256 * 256;
  a.segs = reinterpret_cast<const dtfe::OptSeg*>(blob.data_ptr());
  a.work = reinterpret_cast<const dtfe::OptWork*>((const char*)blob.data_ptr() + off_w);
  a.nwork = (int)nwork;
  if (kind == dtfe::OPT_ADAM) TORCH_CHECK(a.beta_pow && a.s1 && a.s2, "adam needs slots and beta powers");
  if (kind == dtfe::OPT_RMSPROP) TORCH_CHECK(a.s1 && a.s2, "rmsprop needs slots");
  if (kind == dtfe::OPT_MOMENTUM) TORCH_CHECK(a.s1, "momentum needs a slot");
  a.wait_done = g_apply_wait.done; a.wait_seen = g_apply_wait.seen; a.wait_segs = g_apply_wait.segs;
  g_apply_wait = ApplyWait{};
  if (group == 0) {
    TORCH_CHECK(pending.empty(), "apply_gradients: a queued group was never launched");
    dtfe::launch_apply_gradients(a, cur_stream());
    return;
  }
  pending.push_back(a);
  if (group == 2) {
    std::vector<dtfe::OptArgs> q;
    q.swap(pending);
    dtfe::launch_apply_gradients_group(q.data(), (int)q.size(), cur_stream());
  }
}

// ---------------------------------------------------------- elementwise
int data_code(const Tensor& t) {
  if (t.scalar_type() == at::kByte) return 0;
  if (t.scalar_type() == at::kFloat) return 1;
  if (t.scalar_type() == at::kBFloat16) return 2;
  TORCH_CHECK(false, "gather_rows: unsupported dtype");
}

void wgrad_tallk(const Tensor& A, int64_t lda, const Tensor& B, int64_t ldb, int64_t M, int64_t N, int64_t K,
                 const Tensor& out, int64_t ldc, const optional<Tensor>& bias, const Tensor& ws, int64_t splits,
                 double scale) {
  check_cuda(A, "A");
  check_cuda(B, "B");
  check_cuda(out, "out");
  TORCH_CHECK(A.scalar_type() == at::kFloat && B.scalar_type() == at::kFloat && out.scalar_type() == at::kFloat &&
                  ws.scalar_type() == at::kFloat,
              "wgrad_tallk: fp32 operands / output / workspace");
  TORCH_CHECK(A.numel() >= (K - 1) * lda + M && B.numel() >= (K - 1) * ldb + N && out.numel() >= (M - 1) * ldc + N,
              "wgrad_tallk: operand / output extents");
  TORCH_CHECK(ws.numel() >= dtfe::tallk_ws_floats((int)M, (int)N, (int)splits), "wgrad_tallk: workspace too small");
  if (bias) TORCH_CHECK(bias->scalar_type() == at::kFloat && bias->numel() >= N, "wgrad_tallk: bias [N] fp32");
  dtfe::TallKArgs a{};
  a.A = A.data_ptr<float>(); a.lda = (int)lda;
  a.B = B.data_ptr<float>(); a.ldb = (int)ldb;
  a.M = (int)M; a.N = (int)N; a.K = (int)K;
  a.out = out.data_ptr<float>(); a.ldc = (int)ldc;
  a.bias = bias ? bias->data_ptr<float>() : nullptr;
  a.ws = ws.data_ptr<float>(); a.splits = (int)splits;
  a.scale = (float)scale;
  dtfe::launch_wgrad_tallk(a, cur_stream());
}

dtfe::SeqStageArgs seq_stage_args(const Tensor& x, const Tensor& xh, int64_t T, int64_t I, const Tensor& ysrc,
                                   const Tensor& ydst, at::TensorList zero) {
  check_cuda(x, "x");
  check_cuda(xh, "xh");
  TORCH_CHECK(x.scalar_type() == at::kFloat && xh.scalar_type() == at::kFloat && x.is_contiguous() &&
                  xh.is_contiguous() && xh.dim() == 3 && xh.size(0) == T && xh.size(2) > I,
              "seq_stage: x f32 [B][T*I], xh f32 [T][B][ld > I] contiguous");
  const int64_t B = xh.size(1);
  TORCH_CHECK(x.numel() == B * T * I, "seq_stage: x holds B*T*I floats");
  TORCH_CHECK(ysrc.scalar_type() == at::kFloat && ydst.scalar_type() == at::kFloat && ysrc.is_contiguous() &&
                  ydst.is_contiguous() && ysrc.numel() == ydst.numel() && ysrc.numel() % B == 0,
              "seq_stage: label rows f32 [B][*], same size, contiguous");
  dtfe::SeqStageArgs a{};
  a.x = x.data_ptr<float>();
  a.xh = xh.data_ptr<float>();
  a.B = (int)B; a.T = (int)T; a.I = (int)I; a.ld = (int)xh.size(2);
  a.ysrc = ysrc.data_ptr<float>(); a.ydst = ydst.data_ptr<float>(); a.ny = ysrc.numel();
  TORCH_CHECK(zero.size() <= 4, "seq_stage: at most 4 zero ranges");
  for (const Tensor& z : zero) {
    check_cuda(z, "zero");
    TORCH_CHECK(z.is_contiguous() && (z.numel() * z.element_size()) % 4 == 0, "seq_stage: zero ranges must be "
                "contiguous whole 32-bit words");
    a.zptr[a.nz] = reinterpret_cast<uint32_t*>(z.data_ptr());
    a.zlen[a.nz++] = z.numel() * z.element_size() / 4;
  }
  return a;
}

void seq_stage(const Tensor& x, const Tensor& xh, int64_t T, int64_t I, const Tensor& ysrc, const Tensor& ydst,
               at::TensorList zero) {
  dtfe::launch_seq_stage(seq_stage_args(x, xh, T, I, ysrc, ydst, zero), cur_stream());
}

void gather_rows(const Tensor& src, const Tensor& dst, const optional<Tensor>& idx, const optional<Tensor>& labels_src,
                 const optional<Tensor>& labels_dst, int64_t seed, const optional<Tensor>& counter,
                 const optional<Tensor>& done, at::TensorList zero, const optional<Tensor>& onehot) {
  check_cuda(src, "src");
  dtfe::GatherArgs a{};
  if (onehot.has_value()) {
    check_cuda(*onehot, "onehot");
    TORCH_CHECK(onehot->scalar_type() == at::kFloat && onehot->is_contiguous() && onehot->dim() == 2 &&
                onehot->size(0) == dst.size(0) && labels_src.has_value(),
                "gather_rows: onehot must be contiguous f32 [B][ncls] and needs labels_src");
    a.onehot = onehot->data_ptr<float>();
    a.ncls = (int)onehot->size(1);
  }
  TORCH_CHECK(zero.size() <= 4, "gather_rows: at most 4 zero ranges");
  for (const Tensor& z : zero) {
    check_cuda(z, "zero");
    TORCH_CHECK(z.is_contiguous() && (z.numel() * z.element_size()) % 4 == 0, "gather_rows: zero ranges must be "
                "contiguous whole 32-bit words");
    a.zptr[a.nz] = reinterpret_cast<uint32_t*>(z.data_ptr());
    a.zlen[a.nz++] = (long)(z.numel() * z.element_size() / 4);
  }
  a.src = src.data_ptr(); a.src_dtype = data_code(src); a.n_rows = src.size(0); a.D = (int)(src.numel() / src.size(0));
  a.dst = dst.data_ptr(); a.dst_dtype = data_code(dst); a.B = (int)dst.size(0);
  TORCH_CHECK(a.dst_dtype != 0, "gather_rows: dst must be f32 or bf16");
  a.idx = ptr_or_null<int32_t>(idx);
  a.labels_src = ptr_or_null<int32_t>(labels_src); a.labels_dst = ptr_or_null<int32_t>(labels_dst);
  a.seed = (uint64_t)seed; a.counter = ptr_or_null<int64_t>(counter); a.done = ptr_or_null<uint32_t>(done);
  dtfe::launch_gather_rows(a, cur_stream());
}

void uniform_fill(const Tensor& out, double lo, double hi, int64_t seed, const optional<Tensor>& counter,
                  const optional<Tensor>& done, const optional<Tensor>& copy_src, const optional<Tensor>& copy_dst) {
  check_cuda(out, "out");
  const float* cs = nullptr;
  float* cd = nullptr;
  long nc = 0;
  if (copy_src.has_value() && copy_src->defined()) {
    TORCH_CHECK(copy_dst.has_value() && copy_dst->defined(), "uniform_fill: copy_src without copy_dst");
    TORCH_CHECK(copy_src->scalar_type() == at::kFloat && copy_dst->scalar_type() == at::kFloat &&
                    copy_src->is_contiguous() && copy_dst->is_contiguous() && copy_src->numel() == copy_dst->numel() &&
                    copy_src->numel() % 4 == 0 && ((uintptr_t)copy_src->data_ptr() & 15) == 0 &&
                    ((uintptr_t)copy_dst->data_ptr() & 15) == 0,
                "uniform_fill: the fused copy takes equal-size contiguous 16-B aligned fp32 tensors (numel % 4 == 0)");
    cs = copy_src->data_ptr<float>();
    cd = copy_dst->data_ptr<float>();
    nc = copy_src->numel();
  }
  dtfe::launch_uniform_fill(out.data_ptr<float>(), out.numel(), (float)lo, (float)hi, (uint64_t)seed,
                            ptr_or_null<int64_t>(counter), ptr_or_null<uint32_t>(done), cur_stream(), cs, cd, nc);
}

void cast_(const Tensor& src, const Tensor& dst) {
  check_cuda(src, "src");
  TORCH_CHECK(src.numel() == dst.numel(), "cast: size mismatch");
  if (src.scalar_type() == at::kFloat && dst.scalar_type() == at::kBFloat16)
    dtfe::launch_cast_f32_bf16(src.data_ptr<float>(), reinterpret_cast<dtfe::bf16*>(dst.data_ptr()), src.numel(),
                               cur_stream());
  else if (src.scalar_type() == at::kBFloat16 && dst.scalar_type() == at::kFloat)
    dtfe::launch_cast_bf16_f32(reinterpret_cast<const dtfe::bf16*>(src.data_ptr()), dst.data_ptr<float>(),
                               src.numel(), cur_stream());
  else
    TORCH_CHECK(false, "cast: f32<->bf16 only");
}

void softmax_xent(const Tensor& logits, const optional<Tensor>& labels_i, const optional<Tensor>& labels_oh,
                  double scale, const optional<Tensor>& dlogits, const optional<Tensor>& loss_rows,
                  const optional<Tensor>& loss_sum, const optional<Tensor>& correct, const optional<Tensor>& probs) {
  check_cuda(logits, "logits");
  dtfe::XentArgs a{};
  a.B = (int)logits.size(0); a.NC = (int)logits.size(1);
  a.logits = logits.data_ptr<float>();
  a.labels_i = ptr_or_null<int32_t>(labels_i); a.labels_oh = ptr_or_null<float>(labels_oh);
  TORCH_CHECK(a.labels_i || a.labels_oh, "softmax_xent: labels required");
  a.scale = (float)scale;
  a.dlogits = ptr_or_null<float>(dlogits); a.loss_rows = ptr_or_null<float>(loss_rows);
  a.loss_sum = ptr_or_null<float>(loss_sum); a.correct = ptr_or_null<int32_t>(correct);
  a.probs = ptr_or_null<float>(probs);
  dtfe::launch_softmax_xent(a, cur_stream());
}

bool dense_head(const Tensor& feat, const Tensor& w, const optional<Tensor>& bias, const Tensor& y,
                const optional<Tensor>& logits, const optional<Tensor>& loss_sum, const optional<Tensor>& correct,
                const Tensor& dw, const optional<Tensor>& db, const optional<Tensor>& dfeat, double scale,
                bool w_fmajor, bool store, const optional<Tensor>& dl_out) {
  check_cuda(feat, "feat");
  const bool f32 = feat.scalar_type() == at::kFloat;
  TORCH_CHECK((f32 || feat.scalar_type() == at::kBFloat16) && feat.dim() == 2 && feat.is_contiguous(),
              "dense_head: bf16 / fp32 feat [B][F]");
  const int64_t B = feat.size(0), F = feat.size(1), NC = w_fmajor ? w.size(1) : w.size(0);
  TORCH_CHECK(w.scalar_type() == at::kFloat && w.dim() == 2 && w.numel() == NC * F, "dense_head: fp32 w [NC][F] / [F][NC]");
  TORCH_CHECK(y.scalar_type() == at::kFloat && y.numel() == B * NC, "dense_head: fp32 one-hot y [B][NC]");
  TORCH_CHECK(dw.scalar_type() == at::kFloat && dw.numel() == NC * F, "dense_head: fp32 dw");
  const bool has_df = dfeat.has_value() && dfeat->defined();
  TORCH_CHECK(!has_df || (dfeat->scalar_type() == feat.scalar_type() && dfeat->numel() == B * F && dfeat->is_contiguous()),
              "dense_head: dfeat of feat's dtype [B][F]");
  TORCH_CHECK(!dl_out.has_value() || !dl_out->defined() ||
                  (dl_out->scalar_type() == at::kFloat && dl_out->numel() == B * NC && dl_out->is_contiguous()),
              "dense_head: dl_out fp32 [B][NC]");
  TORCH_CHECK(!logits.has_value() || !logits->defined() || logits->numel() == B * NC, "dense_head: logits");
  dtfe::DenseHeadArgs a{};
  a.feat = feat.data_ptr();
  a.f32 = f32 ? 1 : 0;
  a.w_fmajor = w_fmajor ? 1 : 0;
  a.store = store ? 1 : 0;
  a.w = w.data_ptr<float>(); a.bias = ptr_or_null<float>(bias); a.y = y.data_ptr<float>();
  a.logits = ptr_or_null<float>(logits); a.loss_sum = ptr_or_null<float>(loss_sum);
  a.correct = ptr_or_null<int32_t>(correct);
  a.dw = dw.data_ptr<float>(); a.db = ptr_or_null<float>(db);
  a.dfeat = has_df ? dfeat->data_ptr() : nullptr;
  a.dl_out = ptr_or_null<float>(dl_out);
  a.B = (int)B; a.F = (int)F; a.NC = (int)NC; a.scale = (float)scale;
  return dtfe::launch_dense_head(a, cur_stream());
}

void gan_loss(const Tensor& d_real, const Tensor& d_fake, const Tensor& gen_loss, const Tensor& disc_loss,
              const Tensor& dz_real_disc, const Tensor& dz_fake_disc, const Tensor& dz_fake_gen, double clamp_eps) {
  check_cuda(d_real, "d_real");
  dtfe::GanLossArgs a{};
  a.B = (int)d_real.numel();
  a.d_real = d_real.data_ptr<float>(); a.d_fake = d_fake.data_ptr<float>();
  a.gen_loss = gen_loss.data_ptr<float>(); a.disc_loss = disc_loss.data_ptr<float>();
  a.dz_real_disc = dz_real_disc.data_ptr<float>(); a.dz_fake_disc = dz_fake_disc.data_ptr<float>();
  a.dz_fake_gen = dz_fake_gen.data_ptr<float>();
  a.clamp_eps = (float)clamp_eps;
  dtfe::launch_gan_loss(a, cur_stream());
}

bool gan_disc_head(const Tensor& d1, const Tensor& w, const optional<Tensor>& b, const optional<Tensor>& p,
                   const optional<Tensor>& dlog, const optional<Tensor>& dlog_g, const Tensor& gw,
                   const optional<Tensor>& gb, const Tensor& dd1, const Tensor& ddf, const Tensor& gen_loss,
                   const Tensor& disc_loss, const Tensor& ws, double clamp_eps) {
  check_cuda(d1, "d1");
  TORCH_CHECK(d1.dim() == 2 && d1.size(0) % 2 == 0 && d1.scalar_type() == at::kFloat && d1.is_contiguous(),
              "gan_disc_head: d1 f32 [2B][DH] contiguous");
  const int B = (int)(d1.size(0) / 2), DH = (int)d1.size(1);
  auto f32 = [](const Tensor& t, int64_t n) { return t.scalar_type() == at::kFloat && t.is_contiguous() && t.numel() == n; };
  TORCH_CHECK(f32(w, DH) && f32(gw, DH) && f32(dd1, 2L * B * DH) && f32(ddf, (int64_t)B * DH) && f32(gen_loss, 1) &&
                  f32(disc_loss, 1), "gan_disc_head: Wd2 / dWd2 [DH], dd1 [2B][DH], ddf [B][DH], scalar losses (f32)");
  TORCH_CHECK(ws.scalar_type() == at::kFloat && ws.is_contiguous() && ws.numel() >= dtfe::gan_head_ws_floats(B, DH),
              "gan_disc_head: ws needs ", dtfe::gan_head_ws_floats(B, DH), " zeroed floats");
  auto opt_f32 = [](const optional<Tensor>& t) -> float* {
    return t.has_value() && t->defined() ? t->data_ptr<float>() : nullptr;
  };
  dtfe::GanHeadArgs a{};
  a.B = B; a.DH = DH;
  a.d1 = d1.data_ptr<float>(); a.w = w.data_ptr<float>(); a.b = opt_f32(b);
  if (p && p->defined()) { TORCH_CHECK(f32(*p, 2L * B), "gan_disc_head: p [2B]"); a.p = p->data_ptr<float>(); }
  if (dlog && dlog->defined()) { TORCH_CHECK(f32(*dlog, 2L * B), "gan_disc_head: dlog [2B]"); a.dlog = dlog->data_ptr<float>(); }
  if (dlog_g && dlog_g->defined()) { TORCH_CHECK(f32(*dlog_g, B), "gan_disc_head: dlog_g [B]"); a.dlog_g = dlog_g->data_ptr<float>(); }
  a.gw = gw.data_ptr<float>(); a.gb = opt_f32(gb);
  a.dd1 = dd1.data_ptr<float>(); a.ddf = ddf.data_ptr<float>();
  a.gen_loss = gen_loss.data_ptr<float>(); a.disc_loss = disc_loss.data_ptr<float>();
  a.clamp_eps = (float)clamp_eps;
  a.ws = ws.data_ptr<float>();
  return dtfe::launch_gan_disc_head(a, cur_stream());
}

int64_t gan_head_ws_floats(int64_t B, int64_t DH) { return dtfe::gan_head_ws_floats((int)B, (int)DH); }

void mse_sigmoid(const Tensor& y, const Tensor& t, const Tensor& loss, const Tensor& dz, const optional<Tensor>& ws) {
  check_cuda(y, "y");
  TORCH_CHECK(y.is_contiguous() && t.is_contiguous() && dz.is_contiguous() && t.numel() == y.numel() &&
                  dz.numel() == y.numel(), "mse_sigmoid: contiguous y / t / dz of one size");
  float* w = nullptr;
  if (ws.has_value() && ws->defined()) {
    TORCH_CHECK(ws->scalar_type() == at::kFloat && ws->numel() >= dtfe::MSE_WS_FLOATS && ws->is_contiguous(),
                "mse_sigmoid: ws f32 [>= ", dtfe::MSE_WS_FLOATS, "], zero-initialised");
    w = ws->data_ptr<float>();
  }
  dtfe::launch_mse_sigmoid(y.data_ptr<float>(), t.data_ptr<float>(), y.numel(), loss.data_ptr<float>(),
                           dz.data_ptr<float>(), cur_stream(), w);
}

void colsum(const Tensor& x, int64_t M, int64_t N, int64_t ld, const Tensor& db, double scale) {
  check_cuda(x, "x");
  dtfe::launch_colsum(x.data_ptr(), x.scalar_type() == at::kFloat, (int)M, (int)N, ld, db.data_ptr<float>(),
                      (float)scale, cur_stream());
}

void act_grad(const Tensor& dy, const Tensor& y, const Tensor& dz, int64_t act) {
  check_cuda(dy, "dy");
  dtfe::launch_act_grad(dy.data_ptr<float>(), y.data_ptr<float>(), dz.data_ptr<float>(), dy.numel(), (int)act,
                        cur_stream());
}

void bias_act(const Tensor& x, const optional<Tensor>& bias, const Tensor& out, int64_t act, double keep,
              int64_t seed, const optional<Tensor>& counter) {
  check_cuda(x, "x");
  dtfe::BiasActArgs a{};
  a.x = x.data_ptr<float>(); a.bias = ptr_or_null<float>(bias);
  a.M = (int)x.size(0); a.N = (int)(x.numel() / x.size(0)); a.act = (int)act;
  a.keep = (float)keep; a.seed = (uint64_t)seed; a.counter = ptr_or_null<int64_t>(counter);
  a.out = out.data_ptr(); a.out_f32 = out.scalar_type() == at::kFloat;
  dtfe::launch_bias_act(a, cur_stream());
}

void lstm_cell_fwd(const Tensor& gates, const Tensor& act, const optional<Tensor>& c_prev, const Tensor& c,
                   const Tensor& h_out, int64_t ld_h, double forget_bias) {
  check_cuda(gates, "gates");
  dtfe::LstmCellArgs a{};
  a.B = (int)c.size(0); a.H = (int)c.size(1);
  a.gates = gates.data_ptr<float>(); a.act = act.data_ptr<float>(); a.c_prev = ptr_or_null<float>(c_prev);
  a.c = c.data_ptr<float>(); a.h_out = h_out.data_ptr<float>(); a.ld_h = ld_h;
  a.forget_bias = (float)forget_bias;
  dtfe::launch_lstm_cell_fwd(a, cur_stream());
}

void lstm_cell_bwd(const Tensor& act, const optional<Tensor>& c_prev, const Tensor& c, const optional<Tensor>& dh,
                   const optional<Tensor>& dh2, const optional<Tensor>& dc_next, const Tensor& dgates,
                   const Tensor& dc_prev) {
  check_cuda(act, "act");
  dtfe::LstmCellArgs a{};
  a.B = (int)c.size(0); a.H = (int)c.size(1);
  a.act = act.data_ptr<float>(); a.c_prev = ptr_or_null<float>(c_prev); a.c = c.data_ptr<float>();
  a.dh = ptr_or_null<float>(dh); a.dh2 = ptr_or_null<float>(dh2); a.dc_next = ptr_or_null<float>(dc_next);
  a.dgates = dgates.data_ptr<float>(); a.dc_prev = dc_prev.data_ptr<float>();
  dtfe::launch_lstm_cell_bwd(a, cur_stream());
}

// whole-sequence LSTM (lstm_seq.hip): returns false when the shape needs the per-step path
bool lstm_seq_fwd(const Tensor& xh, const Tensor& K, const Tensor& bias, double forget_bias, const Tensor& act,
                  const Tensor& c, const Tensor& hT, const optional<Tensor>& xsrc, const optional<Tensor>& ysrc,
                  const optional<Tensor>& ydst, const optional<Tensor>& zero0, const optional<Tensor>& zero1) {
  check_cuda(xh, "xh");
  TORCH_CHECK(xh.dim() == 3 && xh.scalar_type() == at::kFloat && xh.is_contiguous(), "lstm_seq_fwd: xh [T][B][I+H] f32");
  dtfe::LstmSeqArgs a{};
  a.T = (int)xh.size(0); a.B = (int)xh.size(1); a.H = (int)hT.size(1); a.I = (int)xh.size(2) - a.H;
  TORCH_CHECK(K.numel() == (int64_t)(a.I + a.H) * 4 * a.H && bias.numel() == 4 * a.H, "lstm_seq_fwd: K/bias shape");
  TORCH_CHECK(act.numel() == (int64_t)a.T * a.B * 4 * a.H && c.numel() == (int64_t)a.T * a.B * a.H &&
              hT.numel() == (int64_t)a.B * a.H, "lstm_seq_fwd: output shapes");
  a.xh = xh.data_ptr<float>(); a.K = K.data_ptr<float>(); a.bias = bias.data_ptr<float>();
  a.forget_bias = (float)forget_bias; a.act = act.data_ptr<float>(); a.c = c.data_ptr<float>();
  a.hT = hT.data_ptr<float>();
  if (xsrc.has_value() && xsrc->defined()) {  // seq_stage folded into the forward launch
    TORCH_CHECK(ysrc.has_value() && ydst.has_value(), "lstm_seq_fwd: xsrc needs ysrc / ydst");
    std::vector<Tensor> zero;
    for (const optional<Tensor>* z : {&zero0, &zero1})
      if (z->has_value() && (*z)->defined()) zero.push_back(**z);
    a.st = seq_stage_args(*xsrc, xh, a.T, a.I, *ysrc, *ydst, zero);
  }
  return dtfe::launch_lstm_seq_fwd(a, cur_stream());
}

int64_t lstm_status(bool reset) { return dtfe::lstm_split_status(reset); }

bool lstm_seq_bwd(const Tensor& K, const Tensor& act, const Tensor& c, const Tensor& dhT, const Tensor& dg,
                  int64_t I, const optional<Tensor>& dl, const optional<Tensor>& wo) {
  check_cuda(act, "act");
  dtfe::LstmSeqArgs a{};
  a.T = (int)c.size(0); a.B = (int)c.size(1); a.H = (int)c.size(2); a.I = (int)I;
  TORCH_CHECK(K.numel() == (int64_t)(a.I + a.H) * 4 * a.H, "lstm_seq_bwd: K shape");
  TORCH_CHECK(act.numel() == (int64_t)a.T * a.B * 4 * a.H && dg.numel() == act.numel() &&
              dhT.numel() == (int64_t)a.B * a.H, "lstm_seq_bwd: shapes");
  a.K = K.data_ptr<float>(); a.act = act.data_ptr<float>(); a.c = c.data_ptr<float>();
  a.dhT = dhT.data_ptr<float>(); a.dg = dg.data_ptr<float>();
  if (dl.has_value() && dl->defined()) {  // dh_T = dl . W_out^T formed by the kernel (the fused head's dlogits)
    TORCH_CHECK(wo.has_value() && wo->defined() && wo->dim() == 2 && wo->size(0) == a.H && dl->dim() == 2 &&
                    dl->size(0) == a.B && dl->size(1) == wo->size(1) && dl->is_contiguous() && wo->is_contiguous(),
                "lstm_seq_bwd: dl [B][NC] with W_out [H][NC]");
    a.dl = dl->data_ptr<float>(); a.wo = wo->data_ptr<float>(); a.nc = (int)wo->size(1);
  }
  return dtfe::launch_lstm_seq_bwd(a, cur_stream());
}

}  // namespace

// ------------------------------------------------------------------- norm
dtfe::BnArgs bn_common(const Tensor& x, const Tensor& stats, int64_t act) {
  check_cuda(x, "x");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && x.dim() >= 2, "bn: bf16 [..., C] input");
  dtfe::BnArgs a{};
  a.C = (int)x.size(-1);
  a.R = x.numel() / a.C;
  a.x = reinterpret_cast<const dtfe::bf16*>(x.data_ptr());
  TORCH_CHECK(stats.scalar_type() == at::kFloat && stats.numel() == 2 * a.C, "bn: stats [2][C] fp32");
  a.stats = stats.data_ptr<float>();
  a.act = (int)act;
  return a;
}

void bn_stats(const Tensor& x, const Tensor& stats) {
  dtfe::launch_bn_stats(bn_common(x, stats, 0), cur_stream());
}

void bn_apply(const Tensor& x, const Tensor& stats, const Tensor& gamma, const Tensor& beta,
              const optional<Tensor>& mean, const optional<Tensor>& invstd, const optional<Tensor>& moving_mean,
              const optional<Tensor>& moving_var, double eps, double momentum, int64_t act,
              const optional<Tensor>& res, int64_t rstride, int64_t OH, int64_t OW, const Tensor& out,
              const optional<Tensor>& mask_out, const optional<std::vector<Tensor>>& res_bn) {
  dtfe::BnArgs a = bn_common(x, stats, act);
  if (res_bn.has_value() && !res_bn->empty()) {
    // [stats, gamma, beta, mean, invstd, moving_mean, moving_var] of the residual's own BatchNorm
    const auto& r = *res_bn;
    TORCH_CHECK(r.size() == 7 && res.has_value() && res->sizes() == x.sizes(),
                "bn_apply: res_bn = [stats, gamma, beta, mean, invstd, moving_mean, moving_var] of a same-shape raw residual");
    for (const auto& t : r) TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat, "bn_apply: res_bn fp32 tensors");
    a.r_stats = r[0].data_ptr<float>(); a.r_gamma = r[1].data_ptr<float>(); a.r_beta = r[2].data_ptr<float>();
    a.r_mean = r[3].data_ptr<float>(); a.r_invstd = r[4].data_ptr<float>();
    a.r_moving_mean = r[5].data_ptr<float>(); a.r_moving_var = r[6].data_ptr<float>();
  }
  if (mask_out.has_value() && mask_out->defined()) {
    TORCH_CHECK(mask_out->is_cuda() && mask_out->scalar_type() == at::kByte && mask_out->numel() == x.numel() / 8 &&
                    act == 1, "bn_apply: mask_out is a uint8 [R][C/8] ReLU bit mask");
    a.mask_out = mask_out->data_ptr<uint8_t>();
  }
  a.gamma = gamma.data_ptr<float>();
  a.beta = beta.data_ptr<float>();
  a.mean = ptr_or_null<float>(mean);
  a.invstd = ptr_or_null<float>(invstd);
  a.moving_mean = ptr_or_null<float>(moving_mean);
  a.moving_var = ptr_or_null<float>(moving_var);
  a.eps = (float)eps; a.momentum = (float)momentum;
  a.res = ptr_or_null<dtfe::bf16>(res);
  if (a.res) {
    TORCH_CHECK(res->dim() == 4, "bn_apply: residual NHWC");
    a.RH = (int)res->size(1); a.RW = (int)res->size(2); a.RC = (int)res->size(3);
    a.rstride = (int)rstride; a.OH = (int)OH; a.OW = (int)OW;
  }
  TORCH_CHECK(out.numel() == x.numel() && out.scalar_type() == at::kBFloat16, "bn_apply: out");
  a.out = reinterpret_cast<dtfe::bf16*>(out.data_ptr());
  dtfe::launch_bn_apply(a, cur_stream());
}

// inference-mode BatchNorm: out = act(gamma * (x - moving_mean) * rsqrt(moving_var + eps) + beta [+ res])
void bn_infer(const Tensor& x, const Tensor& gamma, const Tensor& beta, const Tensor& moving_mean,
              const Tensor& moving_var, double eps, int64_t act, const optional<Tensor>& res, int64_t rstride,
              int64_t OH, int64_t OW, const Tensor& out) {
  check_cuda(x, "x");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && x.dim() >= 2, "bn_infer: bf16 [..., C] input");
  dtfe::BnArgs a{};
  a.C = (int)x.size(-1);
  a.R = x.numel() / a.C;
  a.x = reinterpret_cast<const dtfe::bf16*>(x.data_ptr());
  a.act = (int)act;
  a.infer = 1;
  TORCH_CHECK(moving_mean.numel() == a.C && moving_var.numel() == a.C, "bn_infer: moving averages [C]");
  a.gamma = gamma.data_ptr<float>();
  a.beta = beta.data_ptr<float>();
  a.moving_mean = moving_mean.data_ptr<float>();
  a.moving_var = moving_var.data_ptr<float>();
  a.eps = (float)eps;
  a.res = ptr_or_null<dtfe::bf16>(res);
  if (a.res) {
    TORCH_CHECK(res->dim() == 4, "bn_infer: residual NHWC");
    a.RH = (int)res->size(1); a.RW = (int)res->size(2); a.RC = (int)res->size(3);
    a.rstride = (int)rstride; a.OH = (int)OH; a.OW = (int)OW;
  }
  TORCH_CHECK(out.numel() == x.numel() && out.scalar_type() == at::kBFloat16, "bn_infer: out");
  a.out = reinterpret_cast<dtfe::bf16*>(out.data_ptr());
  dtfe::launch_bn_apply(a, cur_stream());
}

// the backward's ReLU-mask source: the bf16 forward output, or its uint8 [R][C/8] bit mask (ReLU only)
void set_bwd_y(dtfe::BnArgs& a, const optional<Tensor>& y, const Tensor& x) {
  if (y.has_value() && y->defined() && y->scalar_type() == at::kByte) {
    TORCH_CHECK(y->is_cuda() && y->numel() == x.numel() / 8 && a.act == 1, "bn_bwd: bit mask is uint8 [R][C/8], ReLU");
    a.ymask = y->data_ptr<uint8_t>();
    return;
  }
  a.y = ptr_or_null<dtfe::bf16>(y);
}

void bn_bwd_stats(const Tensor& dy, const optional<Tensor>& y, const Tensor& x, const Tensor& mean,
                  const Tensor& invstd, const Tensor& stats, int64_t act, const optional<Tensor>& gamma,
                  const optional<Tensor>& beta, const optional<std::vector<Tensor>>& res_bn) {
  dtfe::BnArgs a = bn_common(x, stats, act);
  if (res_bn.has_value() && !res_bn->empty()) {
    // [x, mean, invstd, stats] of a projection shortcut's BN: its statistics from the same g
    const auto& r = *res_bn;
    TORCH_CHECK(r.size() == 4 && r[0].sizes() == x.sizes() && r[0].scalar_type() == at::kBFloat16 &&
                    r[1].scalar_type() == at::kFloat && r[2].scalar_type() == at::kFloat &&
                    r[3].scalar_type() == at::kFloat && r[3].numel() == 2 * a.C,
                "bn_bwd_stats: res_bn = [x bf16 (same shape), mean, invstd, stats [2][C]]");
    a.res = reinterpret_cast<const dtfe::bf16*>(r[0].data_ptr());
    a.r_mean = r[1].data_ptr<float>(); a.r_invstd = r[2].data_ptr<float>(); a.r_stats = r[3].data_ptr<float>();
  }
  a.dy = reinterpret_cast<const dtfe::bf16*>(dy.data_ptr());
  set_bwd_y(a, y, x);
  a.gamma = ptr_or_null<float>(gamma);
  a.beta = ptr_or_null<float>(beta);
  TORCH_CHECK(act == 0 || a.y || a.ymask || (act == 1 && a.gamma && a.beta),
              "bn_bwd: the activation gradient needs the forward output (or, for ReLU, gamma and beta)");
  a.mean = mean.data_ptr<float>();
  a.invstd = invstd.data_ptr<float>();
  dtfe::launch_bn_bwd_stats(a, cur_stream());
}

void bn_bwd_apply(const Tensor& dy, const optional<Tensor>& y, const Tensor& x, const Tensor& mean,
                  const Tensor& invstd, const Tensor& gamma, const Tensor& stats, int64_t act, const Tensor& dx,
                  const optional<Tensor>& dres, const optional<Tensor>& dgamma, const optional<Tensor>& dbeta,
                  const optional<Tensor>& beta) {
  dtfe::BnArgs a = bn_common(x, stats, act);
  a.dy = reinterpret_cast<const dtfe::bf16*>(dy.data_ptr());
  set_bwd_y(a, y, x);
  a.beta = ptr_or_null<float>(beta);
  TORCH_CHECK(act == 0 || a.y || a.ymask || (act == 1 && a.beta),
              "bn_bwd: the activation gradient needs the forward output (or, for ReLU, beta)");
  a.mean = mean.data_ptr<float>();
  a.invstd = invstd.data_ptr<float>();
  a.gamma = gamma.data_ptr<float>();
  a.out = reinterpret_cast<dtfe::bf16*>(dx.data_ptr());
  a.dres = ptr_or_null<dtfe::bf16>(dres);
  a.dgamma = ptr_or_null<float>(dgamma);
  a.dbeta = ptr_or_null<float>(dbeta);
  dtfe::launch_bn_bwd_apply(a, cur_stream());
}

void shortcut_grad_add(const Tensor& g, const Tensor& dx, int64_t stride) {
  TORCH_CHECK(g.dim() == 4 && dx.dim() == 4, "shortcut_grad_add: NHWC tensors");
  dtfe::launch_shortcut_grad_add(reinterpret_cast<const dtfe::bf16*>(g.data_ptr()),
                                 reinterpret_cast<dtfe::bf16*>(dx.data_ptr()), (int)g.size(0), (int)g.size(1),
                                 (int)g.size(2), (int)g.size(3), (int)dx.size(1), (int)dx.size(2), (int)dx.size(3),
                                 (int)stride, cur_stream());
}

void gap_fwd(const Tensor& x, const Tensor& y) {
  TORCH_CHECK(x.dim() == 4, "gap_fwd: NHWC input");
  dtfe::launch_gap_fwd(reinterpret_cast<const dtfe::bf16*>(x.data_ptr()), reinterpret_cast<dtfe::bf16*>(y.data_ptr()),
                       (int)x.size(0), (int)(x.size(1) * x.size(2)), (int)x.size(3), cur_stream());
}

void gap_bwd(const Tensor& dy, const Tensor& dx) {
  TORCH_CHECK(dx.dim() == 4, "gap_bwd: NHWC output");
  dtfe::launch_gap_bwd(reinterpret_cast<const dtfe::bf16*>(dy.data_ptr()), reinterpret_cast<dtfe::bf16*>(dx.data_ptr()),
                       (int)dx.size(0), (int)(dx.size(1) * dx.size(2)), (int)dx.size(3), cur_stream());
}

void maxpool3_fwd(const Tensor& x, const Tensor& y, const Tensor& am) {
  TORCH_CHECK(x.dim() == 4 && y.dim() == 4, "maxpool3: NHWC tensors");
  dtfe::launch_maxpool3_fwd(reinterpret_cast<const dtfe::bf16*>(x.data_ptr()), reinterpret_cast<dtfe::bf16*>(y.data_ptr()),
                            am.data_ptr<uint8_t>(), (int)x.size(0), (int)x.size(1), (int)x.size(2), (int)x.size(3),
                            (int)y.size(1), (int)y.size(2), cur_stream());
}

void pool3_bn_bwd(const Tensor& dp, const Tensor& am, const Tensor& x, const Tensor& mean, const Tensor& invstd,
                  const Tensor& gamma, const Tensor& beta, const Tensor& stats, const Tensor& dx,
                  const optional<Tensor>& dgamma, const optional<Tensor>& dbeta) {
  TORCH_CHECK(dp.dim() == 4 && x.dim() == 4 && dx.sizes() == x.sizes() && am.sizes() == dp.sizes() &&
                  am.scalar_type() == at::kByte && dp.scalar_type() == at::kBFloat16 &&
                  dx.scalar_type() == at::kBFloat16 && dp.size(0) == x.size(0) && dp.size(3) == x.size(3),
              "pool3_bn_bwd: dp / am [B][OH][OW][C], x / dx [B][H][W][C]");
  dtfe::BnArgs a = bn_common(x, stats, 1);
  a.dy = reinterpret_cast<const dtfe::bf16*>(dp.data_ptr());
  a.mean = mean.data_ptr<float>();
  a.invstd = invstd.data_ptr<float>();
  a.gamma = gamma.data_ptr<float>();
  a.beta = beta.data_ptr<float>();
  a.out = reinterpret_cast<dtfe::bf16*>(dx.data_ptr());
  a.dgamma = ptr_or_null<float>(dgamma);
  a.dbeta = ptr_or_null<float>(dbeta);
  dtfe::launch_pool3_bn_bwd(a, am.data_ptr<uint8_t>(), (int)x.size(0), (int)x.size(1), (int)x.size(2),
                            (int)dp.size(1), (int)dp.size(2), cur_stream());
}

void bn_relu_pool3(const Tensor& x, const Tensor& stats, const Tensor& gamma, const Tensor& beta,
                   const optional<Tensor>& mean, const optional<Tensor>& invstd, const optional<Tensor>& moving_mean,
                   const optional<Tensor>& moving_var, double eps, double momentum, const Tensor& y,
                   const Tensor& am) {
  TORCH_CHECK(x.dim() == 4 && y.dim() == 4 && am.dim() == 4, "bn_relu_pool3: NHWC tensors");
  TORCH_CHECK(y.scalar_type() == at::kBFloat16 && am.scalar_type() == at::kByte && y.sizes() == am.sizes() &&
                  y.size(0) == x.size(0) && y.size(3) == x.size(3) && y.size(1) == (x.size(1) + 1) / 2 &&
                  y.size(2) == (x.size(2) + 1) / 2, "bn_relu_pool3: y bf16 / am uint8 [B][ceil(H/2)][ceil(W/2)][C]");
  dtfe::BnArgs a = bn_common(x, stats, 1);
  a.gamma = gamma.data_ptr<float>();
  a.beta = beta.data_ptr<float>();
  a.mean = ptr_or_null<float>(mean);
  a.invstd = ptr_or_null<float>(invstd);
  a.moving_mean = ptr_or_null<float>(moving_mean);
  a.moving_var = ptr_or_null<float>(moving_var);
  a.eps = (float)eps; a.momentum = (float)momentum;
  dtfe::launch_bn_relu_pool3(a, reinterpret_cast<dtfe::bf16*>(y.data_ptr()), am.data_ptr<uint8_t>(), (int)x.size(0),
                             (int)x.size(1), (int)x.size(2), (int)y.size(1), (int)y.size(2), cur_stream());
}

void maxpool3_bwd(const Tensor& dy, const Tensor& am, const Tensor& dx) {
  dtfe::launch_maxpool3_bwd(reinterpret_cast<const dtfe::bf16*>(dy.data_ptr()), am.data_ptr<uint8_t>(),
                            reinterpret_cast<dtfe::bf16*>(dx.data_ptr()), (int)dx.size(0), (int)dx.size(1),
                            (int)dx.size(2), (int)dx.size(3), (int)dy.size(1), (int)dy.size(2), cur_stream());
}

TORCH_LIBRARY(dtfe, m) {
  m.def("conv1_gather_fwd(Tensor images, Tensor labels_src, int seed, Tensor(a!) counter, Tensor(b!) done,"
        " Tensor(c!) labels_dst, Tensor(d!) x, Tensor w, Tensor? bias, Tensor(e!) y, Tensor(f!) argmax,"
        " Tensor(g!)[] zero) -> ()");
  m.def("lstm_seq_fwd(Tensor(a!) xh, Tensor K, Tensor bias, float forget_bias, Tensor(b!) act, Tensor(c!) c,"
        " Tensor(d!) hT, Tensor? xsrc=None, Tensor? ysrc=None, Tensor(e!)? ydst=None, Tensor(f!)? zero0=None,"
        " Tensor(g!)? zero1=None) -> bool");
  m.def("lstm_seq_bwd(Tensor K, Tensor act, Tensor c, Tensor dhT, Tensor(a!) dg, int I, Tensor? dl=None,"
        " Tensor? wo=None) -> bool");
  m.def("lstm_status(bool reset=False) -> int", &lstm_status);
  m.def("bn_stats(Tensor x, Tensor(a!) stats) -> ()");
  m.def("bn_infer(Tensor x, Tensor gamma, Tensor beta, Tensor moving_mean, Tensor moving_var, float eps, int act,"
        " Tensor? res, int rstride, int OH, int OW, Tensor(a!) out) -> ()");
  m.def("bn_apply(Tensor x, Tensor stats, Tensor gamma, Tensor beta, Tensor(a!)? mean, Tensor(b!)? invstd,"
        " Tensor(c!)? moving_mean, Tensor(d!)? moving_var, float eps, float momentum, int act, Tensor? res,"
        " int rstride, int OH, int OW, Tensor(e!) out, Tensor(f!)? mask_out=None, Tensor(g!)[]? res_bn=None) -> ()");
  m.def("bn_bwd_stats(Tensor dy, Tensor? y, Tensor x, Tensor mean, Tensor invstd, Tensor(a!) stats, int act,"
        " Tensor? gamma=None, Tensor? beta=None, Tensor(b!)[]? res_bn=None) -> ()");
  m.def("bn_bwd_apply(Tensor dy, Tensor? y, Tensor x, Tensor mean, Tensor invstd, Tensor gamma, Tensor stats,"
        " int act, Tensor(a!) dx, Tensor(b!)? dres, Tensor(c!)? dgamma, Tensor(d!)? dbeta, Tensor? beta=None) -> ()");
  m.def("shortcut_grad_add(Tensor g, Tensor(a!) dx, int stride) -> ()");
  m.def("gap_fwd(Tensor x, Tensor(a!) y) -> ()");
  m.def("gap_bwd(Tensor dy, Tensor(a!) dx) -> ()");
  m.def("maxpool3_fwd(Tensor x, Tensor(a!) y, Tensor(b!) am) -> ()");
  m.def("maxpool3_bwd(Tensor dy, Tensor am, Tensor(a!) dx) -> ()");
  m.def("bn_relu_pool3(Tensor x, Tensor stats, Tensor gamma, Tensor beta, Tensor(a!)? mean, Tensor(b!)? invstd,"
        " Tensor(c!)? moving_mean, Tensor(d!)? moving_var, float eps, float momentum, Tensor(e!) y,"
        " Tensor(f!) am) -> ()");
  m.def("pool3_bn_bwd(Tensor dp, Tensor am, Tensor x, Tensor mean, Tensor invstd, Tensor gamma, Tensor beta,"
        " Tensor(a!) stats, Tensor(b!) dx, Tensor(c!)? dgamma, Tensor(d!)? dbeta) -> ()");
  m.def("lstm_cell_fwd(Tensor gates, Tensor(a!) act, Tensor? c_prev, Tensor(b!) c, Tensor(c!) h_out, int ld_h,"
        " float forget_bias) -> ()");
  m.def("lstm_cell_bwd(Tensor act, Tensor? c_prev, Tensor c, Tensor? dh, Tensor? dh2, Tensor? dc_next,"
        " Tensor(a!) dgates, Tensor(b!) dc_prev) -> ()");
  m.def(
      "gemm(Tensor A, int amode, int lda, Tensor B, int bmode, int ldb, int M, int N, int K, Tensor(a!) out, int ldc,"
      " Tensor? bias, int bias_axis, int act, float alpha, float beta, bool atomic, int splits, int tile,"
      " Tensor? aux, int ld_aux, int aux_act, int b_ones_row, float keep, int seed, Tensor? counter,"
      " Tensor? pooled, Tensor? argmax, int PH, int PW, int PC, Tensor(b!)? out2, int ldc2, bool out2_trans,"
      " Tensor(c!)? bias_out, Tensor(d!)? ws, Tensor(e!)? tile_ctr, int a_ones_row=-1, Tensor? ones=None) -> ()");
  m.def(
      "conv_fwd(Tensor x, Tensor w, Tensor? bias, Tensor(a!) y, Tensor(b!)? argmax, int B, int H, int W, int C,"
      " int Cout, int OH, int OW, int KH, int KW, int stride, int pad, bool pool, int act, Tensor(c!)? bn_stats=None)"
      " -> ()");
  m.def(
      "conv_dgrad(Tensor dy, Tensor wt, Tensor(a!) dx, int B, int H, int W, int C, int Cout, int OH, int OW, int KH,"
      " int KW, int stride, int pad, Tensor? pooled, Tensor? argmax, Tensor? relu_mask, bool accumulate=False,"
      " Tensor? bnb_x=None, Tensor? bnb_y=None, Tensor? bnb_mean=None, Tensor? bnb_invstd=None,"
      " Tensor? bnb_gamma=None, Tensor? bnb_beta=None, Tensor(b!)? bnb_stats=None, int bnb_act=0,"
      " Tensor? acc_src=None, Tensor? acc_mask=None) -> ()");
  m.def(
      "dense_head(Tensor feat, Tensor w, Tensor? bias, Tensor y, Tensor(a!)? logits, Tensor(b!)? loss_sum,"
      " Tensor(c!)? correct, Tensor(d!) dw, Tensor(e!)? db, Tensor(f!)? dfeat, float scale, bool w_fmajor=False,"
      " bool store=False, Tensor(g!)? dl_out=None) -> bool");
  m.def(
      "imgconv(Tensor? src, Tensor? src_pooled, Tensor? src_argmax, Tensor w, Tensor? bias, Tensor(a!) y,"
      " Tensor(b!)? argmax, Tensor? relu_mask, int B, int SH, int SW, int CS, int OH, int OW, int N, int KH, int KW,"
      " int stride, int pad, bool flip_taps, int act, bool pool, int dil=1, Tensor? sc_src=None,"
      " int sc_stride=1, Tensor(e!)? tstamp=None, Tensor(f!)[]? bn_src=None, float bn_eps=0.001,"
      " float bn_momentum=0.99, bool bn_save=False) -> bool");
  m.def(
      "imgwgrad(Tensor src, Tensor? dy, Tensor? dy_pooled, Tensor? dy_argmax, Tensor(a!) dw, Tensor(b!)? db, int B,"
      " int SH, int SW, int CS, int OH, int OW, int N, int KH, int KW, int stride, int pad, float scale, Tensor(c!)? ws=None,"
      " int max_blocks=0, Tensor[]? bn_src=None, float bn_eps=0.001, bool defer=False) -> ()");
  m.def("wgrad_flush() -> int");
  m.def("wgrad_pending() -> int");
  m.def("wgrad_discard() -> int");
  m.def(
      "conv_wgrad(Tensor dz, Tensor x, Tensor(a!) dw, Tensor(b!)? db, int B, int H, int W, int C, int Cout, int OH,"
      " int OW, int KH, int KW, int stride, int pad, float scale) -> ()");
  m.def(
      "head_xent(Tensor h, Tensor w, Tensor? b, Tensor labels, Tensor(a!) dz, Tensor(b!) dl,"
      " Tensor(c!)? loss_sum, Tensor(d!)? correct, Tensor(e!)? logits, float scale, float inv_keep,"
      " Tensor(f!)? step_counter=None, Tensor(g!)? parts=None) -> ()");
  m.def("head_wgrad(Tensor dl, Tensor h, Tensor(a!) dw, Tensor(b!)? db, int nc, float scale, Tensor? parts=None,"
        " Tensor(c!)? loss_sum=None, Tensor(d!)? correct=None) -> ()");
  m.def("gemm_group(Tensor anchor, bool begin) -> ()");
  m.def("opt_pack(Tensor segs, Tensor work, Tensor device_like) -> Tensor");
  m.def(
      "apply_gradients(int kind, Tensor(a!) p, Tensor? g, Tensor? g16, float gscale, Tensor(b!)? s1, Tensor(c!)? s2,"
      " float lr, float beta1, float beta2, float eps, float momentum, float rho, Tensor(d!)? beta_pow,"
      " Tensor(e!)? global_step, int gs_inc, Tensor(f!) done, Tensor blob, int nseg, int nwork, int group=0) -> ()");
  m.def("wgrad_tallk(Tensor A, int lda, Tensor B, int ldb, int M, int N, int K, Tensor(a!) out, int ldc,"
        " Tensor(b!)? bias, Tensor(c!) ws, int splits, float scale) -> ()");
  m.def("seq_stage(Tensor x, Tensor(a!) xh, int T, int I, Tensor ysrc, Tensor(b!) ydst, Tensor(c!)[] zero) -> ()");
  m.def(
      "gather_rows(Tensor src, Tensor(a!) dst, Tensor? idx, Tensor? labels_src, Tensor(b!)? labels_dst, int seed,"
      " Tensor(c!)? counter, Tensor(d!)? done, Tensor(e!)[] zero, Tensor(f!)? onehot=None) -> ()");
  m.def("uniform_fill(Tensor(a!) out, float lo, float hi, int seed, Tensor(b!)? counter, Tensor(c!)? done,"
        " Tensor? copy_src=None, Tensor(d!)? copy_dst=None) -> ()");
  m.def("cast_(Tensor src, Tensor(a!) dst) -> ()");
  m.def(
      "softmax_xent(Tensor logits, Tensor? labels_i, Tensor? labels_oh, float scale, Tensor(a!)? dlogits,"
      " Tensor(b!)? loss_rows, Tensor(c!)? loss_sum, Tensor(d!)? correct, Tensor(e!)? probs) -> ()");
  m.def(
      "gan_loss(Tensor d_real, Tensor d_fake, Tensor(a!) gen_loss, Tensor(b!) disc_loss, Tensor(c!) dz_real_disc,"
      " Tensor(d!) dz_fake_disc, Tensor(e!) dz_fake_gen, float clamp_eps) -> ()");
  m.def("gan_disc_head(Tensor d1, Tensor w, Tensor? b, Tensor(a!)? p, Tensor(b!)? dlog, Tensor(c!)? dlog_g,"
        " Tensor(d!) gw, Tensor(e!)? gb, Tensor(f!) dd1, Tensor(g!) ddf, Tensor(h!) gen_loss, Tensor(i!) disc_loss,"
        " Tensor(j!) ws, float clamp_eps=0.0) -> bool");
  m.def("gan_head_ws_floats(int B, int DH) -> int");
  m.def("apply_wait_next(Tensor done, Tensor seen, int segs) -> ()");
  m.def("epoch_signal(Tensor(a!) ctr) -> ()");
  m.def("mse_sigmoid(Tensor y, Tensor t, Tensor(a!) loss, Tensor(b!) dz, Tensor(c!)? ws=None) -> ()");
  m.def("colsum(Tensor x, int M, int N, int ld, Tensor(a!) db, float scale) -> ()");
  m.def("unpool_f32(Tensor g, Tensor argmax, Tensor(a!) out, int B, int PH, int PW, int C) -> ()");
  m.def("head_xent_f32(Tensor h, Tensor w, Tensor? b, Tensor labels, Tensor(a!) dz, Tensor(b!) dl, Tensor(c!) loss_sum,"
        " Tensor(d!) correct, Tensor(e!)? logits, float scale, float inv_keep, Tensor(f!)? step_counter) -> bool");
  m.def("conv1_wgrad_pooled_f32(Tensor dp, Tensor argmax, Tensor x, Tensor(a!) dw, Tensor(b!)? db, Tensor(c!) ws,"
        " int B, int H, int W, int K, float scale) -> bool");
  m.def("transpose_taps_f32(Tensor input, Tensor(a!) out, int O, int T, int C) -> ()");
  m.def("act_grad(Tensor dy, Tensor y, Tensor(a!) dz, int act) -> ()");
  m.def("bias_act(Tensor x, Tensor? bias, Tensor(a!) out, int act, float keep, int seed, Tensor? counter) -> ()");
}

TORCH_LIBRARY_IMPL(dtfe, CUDA, m) {
  m.impl("conv1_gather_fwd", &conv1_gather_fwd);
  m.impl("lstm_seq_fwd", &lstm_seq_fwd);
  m.impl("lstm_seq_bwd", &lstm_seq_bwd);
  m.impl("bn_stats", &bn_stats);
  m.impl("bn_apply", &bn_apply);
  m.impl("bn_infer", &bn_infer);
  m.impl("bn_bwd_stats", &bn_bwd_stats);
  m.impl("bn_bwd_apply", &bn_bwd_apply);
  m.impl("shortcut_grad_add", &shortcut_grad_add);
  m.impl("gap_fwd", &gap_fwd);
  m.impl("gap_bwd", &gap_bwd);
  m.impl("maxpool3_fwd", &maxpool3_fwd);
  m.impl("maxpool3_bwd", &maxpool3_bwd);
  m.impl("bn_relu_pool3", &bn_relu_pool3);
  m.impl("pool3_bn_bwd", &pool3_bn_bwd);
  m.impl("gemm", &gemm);
  m.impl("conv_fwd", &conv_fwd);
  m.impl("conv_dgrad", &conv_dgrad);
  m.impl("conv_wgrad", &conv_wgrad);
  m.impl("head_xent", &head_xent);
  m.impl("head_wgrad", &head_wgrad);
  m.impl("gemm_group", &gemm_group);
  m.impl("apply_gradients", &apply_gradients);
  m.impl("gather_rows", &gather_rows);
  m.impl("seq_stage", &seq_stage);
  m.impl("wgrad_tallk", &wgrad_tallk);
  m.impl("uniform_fill", &uniform_fill);
  m.impl("cast_", &cast_);
  m.impl("softmax_xent", &softmax_xent);
  m.impl("gan_loss", &gan_loss);
  m.impl("mse_sigmoid", &mse_sigmoid);
  m.impl("gan_disc_head", &gan_disc_head);
  m.impl("apply_wait_next", &apply_wait_next);
  m.impl("epoch_signal", &epoch_signal);
  m.impl("colsum", &colsum);
  m.impl("unpool_f32", &unpool_f32);
  m.impl("head_xent_f32", &head_xent_f32);
  m.impl("conv1_wgrad_pooled_f32", &conv1_wgrad_pooled_f32);
  m.impl("transpose_taps_f32", &transpose_taps_f32);
  m.impl("act_grad", &act_grad);
  m.impl("bias_act", &bias_act);
  m.impl("imgconv", &imgconv);
  m.impl("dense_head", &dense_head);
  m.impl("imgwgrad", &imgwgrad);
  m.impl("lstm_cell_fwd", &lstm_cell_fwd);
  m.impl("lstm_cell_bwd", &lstm_cell_bwd);
}

// every weight-gradient reduce queued with imgwgrad(defer=True), as one grouped launch on the current stream
int64_t wgrad_flush() { return dtfe::flush_wgrad_reduces(cur_stream()); }
int64_t wgrad_pending() { return dtfe::pending_wgrad_reduces(); }
int64_t wgrad_discard() { return dtfe::discard_wgrad_reduces(); }

TORCH_LIBRARY_IMPL(dtfe, CompositeExplicitAutograd, m) {
  m.impl("opt_pack", &opt_pack);
  m.impl("wgrad_flush", &wgrad_flush);
  m.impl("wgrad_pending", &wgrad_pending);
  m.impl("wgrad_discard", &wgrad_discard);
  m.impl("gan_head_ws_floats", &gan_head_ws_floats);
}
