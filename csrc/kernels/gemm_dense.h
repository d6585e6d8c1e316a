// Dense GEMM (fc layers of every model) with a fused epilogue:
//   out = act(alpha * A.B^T + bias) (+ beta * out)     or     atomicAdd(out, A.B^T)
#pragma once
#include "gemm_core.h"
#include "conv.h"

namespace dtfe {

constexpr int GEMM_KTILE = 64;  // k-tile depth of the dense GEMMs (2 MFMA k-steps per barrier)


struct DenseGemmArgs {
  int M, N, K;
  const void* A; long lda;     // A(m,k): KMAJ a[m*lda+k], RMAJ a[k*lda+m]
  const void* B; long ldb;     // B(n,k): KMAJ b[n*ldb+k], RMAJ b[k*ldb+n]
  int b_ones_row;              // >=0: B row that reads as 1.0 (bias column)
  int a_ones_row;              // >=0: A row that reads as 1.0 (bias row: out[a_ones_row][n] -> bias_out[n])
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
  // split-K with a fused (non-atomic) epilogue: every split stores its partial
  // tile to ws[split][tile]; the last split to arrive (tile_ctr) sums them in
  // fixed split order (deterministic), resets the counter and runs the epilogue
  float* ws; int* tile_ctr;
  // global_load_lds kernel (tiles 5..8): a 1 KB page of bf16 ones, read by the whole n-tile that
  // starts at b_ones_row (the bias column of a weight-gradient GEMM sits past the operand's rows)
  const bf16* ones;
};

// Epilogue of one output element (row < M, col < N); returns false when the
// element was fully handled (atomic / bias column / unpool) and x must not be stored.
__device__ __forceinline__ bool dense_epi(const DenseGemmArgs& a, int row, int col, float& x, int64_t drop_step,
                                          float inv_keep) {
  const long o = (long)row * a.ldc + col;
  if (a.bias_out && row == a.a_ones_row) {  // the ones row = this layer's bias gradient (per column)
    if (a.atomic) atomicAdd(a.bias_out + col, a.alpha * x);
    else a.bias_out[col] = a.alpha * x;
    return false;
  }
  if (a.bias_out && col == a.b_ones_row) {  // the ones column = this layer's bias gradient
    if (a.atomic) atomicAdd(a.bias_out + row, a.alpha * x);
    else a.bias_out[row] = a.alpha * x;
    return false;
  }
  if (a.atomic) {
    atomicAdd(reinterpret_cast<float*>(a.out) + o, a.alpha * x);
    return false;
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
    unpool_store(a.up, o, x, reinterpret_cast<bf16*>(a.out));
    return false;
  }
  if (a.beta != 0.f) {
    const float old = a.out_f32 ? reinterpret_cast<float*>(a.out)[o] : bf2f(reinterpret_cast<bf16*>(a.out)[o]);
    x += a.beta * old;
  }
  if (a.out2) {
    const long o2 = a.out2_trans ? (long)col * a.ldc2 + row : (long)row * a.ldc2 + col;
    if (a.out2_f32) reinterpret_cast<float*>(a.out2)[o2] = x;
    else reinterpret_cast<bf16*>(a.out2)[o2] = f2bf(x);
  }
  return true;
}

// Everything after the k-loop: accumulators -> f32 C tile in LDS (the operand buffers are dead,
// the caller has passed a barrier), optional deterministic split-K combine (last arriver), then
// the fused epilogue walking 8-column chunks (coalesced 16-32 B stores).  Shared by the
// register-staged kernel below and the global_load_lds kernel of gemm_glds.h.
template <typename Cfg, int NT = GEMM_THREADS>
__device__ __forceinline__ void dense_epilogue(const DenseGemmArgs& a, char* smem_raw, f32x4_t (&acc)[Cfg::TM][Cfg::TN],
                                               int tm, int tn, int tiles_m, int tiles_n) {
  constexpr int CLD = Cfg::BN + 4;  // f32 C tile row stride: 16*(odd) bytes, conflict-free quad writes
  float* Cs = reinterpret_cast<float*>(smem_raw);
  const int m_base = tm * Cfg::BM, n_base = tn * Cfg::BN;
  // (k-group kernels: NT > 256 threads, the first 4 waves hold the folded tile; the 8-wave fc tile: all 8)
  if (NT == Cfg::WAVES * 64 || threadIdx.x < Cfg::WAVES * 64) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int wm = wid / Cfg::WARPS_N, wn = wid % Cfg::WARPS_N;
#pragma unroll
    for (int i = 0; i < Cfg::TM; ++i)
#pragma unroll
      for (int j = 0; j < Cfg::TN; ++j) {
        const int r = wm * Cfg::WM + i * 16 + (lane >> 4) * 4, c = wn * Cfg::WN + j * 16 + (lane & 15);
#pragma unroll
        for (int q = 0; q < 4; ++q) Cs[(r + q) * CLD + c] = acc[i][j][q];
      }
  }
  __syncthreads();
  constexpr int CPR = Cfg::BN / 8;              // 8-column chunks per row
  constexpr int NCH = Cfg::BM * CPR;            // chunks per tile
  if (gridDim.z > 1 && !a.atomic) {
    // deterministic split-K: partial tile -> ws[z][tile], the last split to arrive sums in split order
    const int tile = tm * tiles_n + tn, ntiles = tiles_m * tiles_n;
    float* mine = a.ws + ((long)blockIdx.z * ntiles + tile) * (Cfg::BM * Cfg::BN);
    // hand-off (MI355X guide, split-K counter form with write-through slabs): the slab leaves in
    // 16-B sc1 (write-through) buffer stores, every wave drains them, barrier, ONE lane takes a
    // ticket with a relaxed agent-scope add - no release fence (an agent-scope release writes the
    // XCD's dirty L2 lines back; one per split workgroup made the MNIST fc1 split-K GEMMs 2-4x
    // SLOWER than no split, profiles/r2_fc1_gemm_sweep.txt); the last arriver acquires once and
    // reads every slab.  Valid on gfx950 (MI355X), the only ARCH this library builds for (csrc/build.py):
    // sc1 buffer stores write through the XCD's L2 there, which is what makes the drained slab
    // visible to a last arriver on another XCD without a release (MI355X_MICROARCH.md, valid forms);
    // tests/test_kernels_gpu.py::test_splitk_combine_many_splits_deterministic pins it.
    const __amdgpu_buffer_rsrc_t slab = __builtin_amdgcn_make_buffer_rsrc(mine, (short)0, Cfg::BM * Cfg::BN * 4, 0x00020000);
    for (int ch = threadIdx.x; ch < NCH; ch += NT) {
      const int r = ch / CPR, c = (ch % CPR) * 8;
      __builtin_amdgcn_raw_buffer_store_b128(*reinterpret_cast<const u32x4_t*>(Cs + r * CLD + c), slab, ch * 32, 0, 16);
      __builtin_amdgcn_raw_buffer_store_b128(*reinterpret_cast<const u32x4_t*>(Cs + r * CLD + c + 4), slab, ch * 32 + 16, 0,
                                             16);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int* flag = reinterpret_cast<int*>(smem_raw);  // the one LDS array (Cs is free here)
    if (threadIdx.x == 0) {
      const int prev = __hip_atomic_fetch_add(a.tile_ctr + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = prev == (int)gridDim.z - 1;
      if (last) {
        __hip_atomic_store(a.tile_ctr + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // next launch / replay
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      *flag = last;
    }
    __syncthreads();
    const int last = *flag;
    __syncthreads();
    if (!last) return;
    for (int ch = threadIdx.x; ch < NCH; ch += NT) {
      const int r = ch / CPR, c = (ch % CPR) * 8;
      f32x4_t v0 = {0.f, 0.f, 0.f, 0.f}, v1 = v0;
      for (int z = 0; z < (int)gridDim.z; ++z) {
        const f32x4_t* src = reinterpret_cast<const f32x4_t*>(a.ws + ((long)z * ntiles + tile) * (Cfg::BM * Cfg::BN) + ch * 8);
        v0 += src[0];
        v1 += src[1];
      }
      *reinterpret_cast<f32x4_t*>(Cs + r * CLD + c) = v0;
      *reinterpret_cast<f32x4_t*>(Cs + r * CLD + c + 4) = v1;
    }
    __syncthreads();
  }
  const int64_t drop_step = (a.keep < 1.f && a.counter) ? *a.counter : 0;
  const float inv_keep = 1.f / a.keep;
  // plain-store fast path: no per-element side outputs, 16 B aligned rows
  // (a weight-gradient GEMM's bias row / column only takes the per-element path in its own chunks)
  const bool vec_store = !a.atomic && !a.unpool && !a.out2 && a.beta == 0.f &&
                         (a.ldc % 8) == 0 && ((((uintptr_t)a.out) & 15) == 0);
  for (int ch = threadIdx.x; ch < NCH; ch += NT) {
    const int r = ch / CPR, c = (ch % CPR) * 8;
    const int row = m_base + r, col0 = n_base + c;
    if (row >= a.M || col0 >= a.N) continue;
    float x[8];
    *reinterpret_cast<f32x4_t*>(x) = *reinterpret_cast<const f32x4_t*>(Cs + r * CLD + c);
    *reinterpret_cast<f32x4_t*>(x + 4) = *reinterpret_cast<const f32x4_t*>(Cs + r * CLD + c + 4);
    const bool side = a.bias_out && (row == a.a_ones_row || (a.b_ones_row >= col0 && a.b_ones_row < col0 + 8));
    if (vec_store && !side && col0 + 8 <= a.N) {
      const long o = (long)row * a.ldc + col0;
      float g[8];  // act'(aux) factors, one 16 B load when aux is bf16 and aligned
      if (a.aux && !a.aux_f32 && (a.ld_aux % 8) == 0) {
        const u32x4_t av = *reinterpret_cast<const u32x4_t*>(reinterpret_cast<const bf16*>(a.aux) +
                                                              (long)row * a.ld_aux + col0);
#pragma unroll
        for (int e = 0; e < 8; ++e) g[e] = act_grad_from_out(bf2f((bf16)(av[e >> 1] >> (16 * (e & 1)))), a.aux_act);
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          float y = 1.f;
          if (a.aux) {
            const long oa = (long)row * a.ld_aux + col0 + e;
            y = act_grad_from_out(a.aux_f32 ? reinterpret_cast<const float*>(a.aux)[oa]
                                            : bf2f(reinterpret_cast<const bf16*>(a.aux)[oa]), a.aux_act);
          }
          g[e] = y;
        }
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float v = x[e] * a.alpha;
        if (a.bias) v += a.bias[a.bias_axis ? row : col0 + e];
        v = apply_act(v, a.act);
        if (a.keep < 1.f)
          v = hash_uniform(a.seed, (uint64_t)drop_step * ((uint64_t)a.M * a.N) + (uint64_t)(o + e)) < a.keep ? v * inv_keep
                                                                                                         : 0.f;
        x[e] = v * g[e];
      }
      if (a.out_f32) {
        reinterpret_cast<f32x4_t*>(reinterpret_cast<float*>(a.out) + o)[0] = *reinterpret_cast<f32x4_t*>(x);
        reinterpret_cast<f32x4_t*>(reinterpret_cast<float*>(a.out) + o)[1] = *reinterpret_cast<f32x4_t*>(x + 4);
      } else {
        u32x4_t v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = pack_bf16x2(x[2 * e], x[2 * e + 1]);
        *reinterpret_cast<u32x4_t*>(reinterpret_cast<bf16*>(a.out) + o) = v;
      }
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int col = col0 + e;
        if (col >= a.N) break;
        float xe = x[e];
        if (!dense_epi(a, row, col, xe, drop_step, inv_keep)) continue;
        const long o = (long)row * a.ldc + col;
        if (a.out_f32) reinterpret_cast<float*>(a.out)[o] = xe;
        else reinterpret_cast<bf16*>(a.out)[o] = f2bf(xe);
      }
    }
  }
}

template <typename Cfg> struct DenseCBytes { static constexpr int VALUE = Cfg::BM * (Cfg::BN + 4) * 4; };

template <typename T, typename Cfg, int AMODE, int BMODE>
__global__ __launch_bounds__(GEMM_THREADS) void gemm_dense_kernel(DenseGemmArgs a) {
  using LA = DenseLoader<T, Cfg::BM, AMODE, Cfg::BK>;
  using LB = DenseLoader<T, Cfg::BN, BMODE, Cfg::BK>;
  constexpr int SMEM_BYTES = SmemSize<T, Cfg, LA, LB>::BYTES > DenseCBytes<Cfg>::VALUE ? SmemSize<T, Cfg, LA, LB>::BYTES
                                                                                      : DenseCBytes<Cfg>::VALUE;
  __shared__ __attribute__((aligned(16))) char smem_raw[SMEM_BYTES];
  T* smem = reinterpret_cast<T*>(smem_raw);
  const int tiles_m = (a.M + Cfg::BM - 1) / Cfg::BM, tiles_n = (a.N + Cfg::BN - 1) / Cfg::BN;
  int tm, tn;
  tile_coords(tiles_m, tiles_n, tm, tn);
  const int m_base = tm * Cfg::BM, n_base = tn * Cfg::BN;
  const int k_begin = blockIdx.z * a.k_chunk;
  const int k_end = min(a.K, k_begin + a.k_chunk);
  LA la((const T*)a.A, a.lda, a.M, a.K, m_base, a.a_ones_row);
  LB lb((const T*)a.B, a.ldb, a.N, a.K, n_base, a.b_ones_row);
  f32x4_t acc[Cfg::TM][Cfg::TN];
  gemm_mainloop<T, Cfg, AMODE, BMODE>(la, lb, k_begin, k_end, smem, acc);  // ends with a barrier
  dense_epilogue<Cfg>(a, smem_raw, acc, tm, tn, tiles_m, tiles_n);
}

// host-side launcher (defined in gemm_dense.hip)
// dtype: 0 = bf16, 1 = f32.  tile: 0 = 64x64, 1 = 128x128, 2 = 128x64, 3 = 64x128, 4 = 32x32
// (register-staged engine of gemm_core.h); 5 = 128x128, 6 = 128x64, 7 = 64x128, 8 = 64x64 with
// direct global->LDS staging, 3 stages (gemm_glds.h: bf16, K % 64 == 0, whole tiles - see
// gemm_glds_eligible); 9..12 the same tiles with 2 stages; 14..16 64x64 with 4 / 6 / 8 stages,
// 19..21 64x64 with 2 / 4 / 2 in-workgroup k-groups,
// 17..18 128x64 with 4 / 6 stages
void launch_gemm_dense(int dtype, int amode, int bmode, int tile, int splits, const DenseGemmArgs& args,
                       hipStream_t stream);
// tile 13: exact-fp32 16x16 tiles, one workgroup per tile with an in-workgroup 4-way K split and
// register-direct operands (gemm_small.hip) - the small layers of the reference workloads
constexpr int GEMM_TILE_SMALL = 13;
bool gemm_small_eligible(int dtype, const DenseGemmArgs& a);
void launch_gemm_small(int amode, int bmode, const DenseGemmArgs& a, hipStream_t s);
// n (<= 2) small GEMMs recorded inside a gemm group: a (RMAJ, RMAJ) + (KMAJ, KMAJ) pair leaves as one
// launch, anything else launches one by one in recording order
void launch_gemm_small_group(int n, const int* am, const int* bm, const DenseGemmArgs* g, hipStream_t s);
// Grouped launch (gemm_dense.hip): between begin and end, launch_gemm_dense calls with glds tile 12
// or 22 (both pieces the same tile) and one split, and launch_head_wgrad calls, are recorded instead of launched (record functions
// return false when a call does not fit the group); end launches the recorded pieces as one grid
// (head weight gradient, then a (KMAJ, RMAJ) and a (RMAJ, RMAJ) GEMM), or one by one otherwise.
struct HeadWgradArgs;
void glds_group_begin();
bool glds_group_record(int amode, int bmode, int tile, const DenseGemmArgs& a);
bool glds_group_record_head(const HeadWgradArgs& a);
void glds_group_end(hipStream_t s);
// block tile of a tile id; returns the k-tile depth (split-K chunks are multiples of it)
int gemm_dense_tile_dims(int tile, int& bm, int& bn);
// whether the global_load_lds kernel family can run this GEMM with tile `tile` (5..8)
bool gemm_glds_eligible(int dtype, int amode, int bmode, int tile, const DenseGemmArgs& a);

}  // namespace dtfe
