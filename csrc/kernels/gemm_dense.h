// Dense GEMM (fc layers of every model) with a fused epilogue:
//   out = act(alpha * A.B^T + bias) (+ beta * out)     or     atomicAdd(out, A.B^T)
#pragma once
#include "gemm_core.h"
#include "conv.h"

namespace dtfe {

struct DenseGemmArgs {
  int M, N, K;
  const void* A; long lda;     // A(m,k): KMAJ a[m*lda+k], RMAJ a[k*lda+m]
  const void* B; long ldb;     // B(n,k): KMAJ b[n*ldb+k], RMAJ b[k*ldb+n]
  int b_ones_row;              // >=0: B row that reads as 1.0 (bias column)
  int k_chunk;                 // split-K chunk (multiple of BK); gridDim.z splits
  // epilogue
  void* out; long ldc; int out_f32;
  const float* bias; int bias_axis;  // 0: bias[n], 1: bias[m]
  int act; float alpha; float beta; int atomic;
  // optional: second output receiving the same values (e.g. f32 copy), may be null
  void* out2; long ldc2; int out2_f32; int out2_trans;  // out2_trans: store at [n*ldc2+m]
  // fused activation-gradient prologue of the backward pass:
  // x *= act'(aux[m][n]) where aux holds the forward OUTPUT of the activation
  const void* aux; long ld_aux; int aux_f32; int aux_act;
  // fused un-pool epilogue (CNN fc1 dgrad): bf16 output routed through argmax
  int unpool; UnpoolArgs up;
  // fused dropout after the activation: keep with prob `keep` (hash RNG of
  // (seed, *counter, element)), scale kept values by 1/keep
  float keep; uint64_t seed; const int64_t* counter;
  // weight-gradient GEMMs: column b_ones_row (B row of ones) is routed to bias_out[m]
  float* bias_out;
};

template <typename T, typename Cfg, int AMODE, int BMODE>
__global__ __launch_bounds__(GEMM_THREADS) void gemm_dense_kernel(DenseGemmArgs a) {
  using LA = DenseLoader<T, Cfg::BM, AMODE>;
  using LB = DenseLoader<T, Cfg::BN, BMODE>;
  __shared__ __attribute__((aligned(16))) T smem[SmemSize<T, Cfg, LA, LB>::ELEMS];
  const int tiles_m = (a.M + Cfg::BM - 1) / Cfg::BM, tiles_n = (a.N + Cfg::BN - 1) / Cfg::BN;
  int tm, tn;
  tile_coords(tiles_m, tiles_n, tm, tn);
  const int m_base = tm * Cfg::BM, n_base = tn * Cfg::BN;
  const int k_begin = blockIdx.z * a.k_chunk;
  const int k_end = min(a.K, k_begin + a.k_chunk);
  LA la((const T*)a.A, a.lda, a.M, a.K, m_base, -1);
  LB lb((const T*)a.B, a.ldb, a.N, a.K, n_base, a.b_ones_row);
  f32x4_t acc[Cfg::TM][Cfg::TN];
  gemm_mainloop<T, Cfg, AMODE, BMODE>(la, lb, k_begin, k_end, smem, acc);
  const int64_t drop_step = (a.keep < 1.f && a.counter) ? *a.counter : 0;
  const float inv_keep = 1.f / a.keep;

  for_each_quad<Cfg>(m_base, n_base, acc, [&](int row0, int col, f32x4_t v) {
    if (col >= a.N) return;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int row = row0 + j;
      if (row >= a.M) continue;
      float x = v[j];
      const long o = (long)row * a.ldc + col;
      if (a.bias_out && col == a.b_ones_row) {  // the ones column = this layer's bias gradient
        if (a.atomic) atomicAdd(a.bias_out + row, a.alpha * x);
        else a.bias_out[row] = a.alpha * x;
        continue;
      }
      if (a.atomic) {
        atomicAdd(reinterpret_cast<float*>(a.out) + o, a.alpha * x);
        continue;
      }
      x *= a.alpha;
      if (a.bias) x += a.bias[a.bias_axis ? row : col];
      x = apply_act(x, a.act);
      if (a.keep < 1.f)
        x = hash_uniform(a.seed, (uint64_t)drop_step * ((uint64_t)a.M * a.N) + (uint64_t)o) < a.keep ? x * inv_keep : 0.f;
      if (a.aux) {
        const long oa = (long)row * a.ld_aux + col;
        const float y = a.aux_f32 ? reinterpret_cast<const float*>(a.aux)[oa] : bf2f(reinterpret_cast<const bf16*>(a.aux)[oa]);
        x *= act_grad_from_out(y, a.aux_act);
      }
      if (a.unpool) {
        unpool_store(a.up, (long)row * a.ldc + col, x, reinterpret_cast<bf16*>(a.out));
        continue;
      }
      if (a.beta != 0.f) {
        const float old = a.out_f32 ? reinterpret_cast<float*>(a.out)[o] : bf2f(reinterpret_cast<bf16*>(a.out)[o]);
        x += a.beta * old;
      }
      if (a.out_f32) reinterpret_cast<float*>(a.out)[o] = x;
      else reinterpret_cast<bf16*>(a.out)[o] = f2bf(x);
      if (a.out2) {
        const long o2 = a.out2_trans ? (long)col * a.ldc2 + row : (long)row * a.ldc2 + col;
        if (a.out2_f32) reinterpret_cast<float*>(a.out2)[o2] = x;
        else reinterpret_cast<bf16*>(a.out2)[o2] = f2bf(x);
      }
    }
  });
}

// host-side launcher (defined in gemm_dense_*.hip)
// dtype: 0 = bf16, 1 = f32.  tile: 0 = 64x64, 1 = 128x128, 2 = 128x64, 3 = 64x128, 4 = 32x32
void launch_gemm_dense(int dtype, int amode, int bmode, int tile, int splits, const DenseGemmArgs& args,
                       hipStream_t stream);

}  // namespace dtfe
