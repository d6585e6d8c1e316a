// Fused multi-tensor apply_gradients: one launch updates
// every parameter of a model in the flat fp32 master buffer with TF1-exact
// math, refreshes the bf16 working copies the MFMA kernels read (natural and,
// where a backward GEMM wants it, transposed through an LDS tile), and - in
// its last workgroup - advances global_step and Adam's beta powers, the
// scalars TF keeps as separate variables (AssignAdd / _finish in TF1).
//
// TF1 reference semantics (tensorflow/python/training/*.py @ 1.11):
//   SGD       : v -= lr*g
//   Momentum  : a = m*a + g ; v -= lr*a
//   Adam      : lr_t = lr*sqrt(1-b2^t)/(1-b1^t); m = b1 m + (1-b1) g;
//               v2 = b2 v2 + (1-b2) g^2; v -= lr_t * m / (sqrt(v2) + eps)
//   RMSProp   : ms = rho ms + (1-rho) g^2 ; mom = mu mom + lr g / sqrt(ms + eps); v -= mom
//               (ms slot initialised to ONES by the host)
//
// Memory-bound: the flat path moves 4 elements per thread per iteration with
// 16-byte loads/stores of every stream (p, g, slots) and 8-byte bf16 stores.
#include "optim.h"

namespace dtfe {

template <int KIND>
__device__ __forceinline__ float upd(const OptArgs& a, float lr_t, float v, float g, float& s1, float& s2) {
  // no multiply-add contraction: the rounding of every update must not depend on how a kernel
  // instantiation's instruction selection happened to fuse it (a grouped launch of several
  // optimizers and separate launches must agree bitwise)
#pragma clang fp contract(off)
  if constexpr (KIND == OPT_SGD) {
    return v - a.lr * g;
  } else if constexpr (KIND == OPT_MOMENTUM) {
    s1 = s1 * a.momentum + g;
    return v - a.lr * s1;
  } else if constexpr (KIND == OPT_ADAM) {
    return tf1_adam(v, g, s1, s2, lr_t, a.beta1, a.beta2, a.eps);
  } else {
    s1 = s1 * a.rho + (1.f - a.rho) * g * g;
    s2 = s2 * a.momentum + a.lr * g / sqrtf(s1 + a.eps);
    return v - s2;
  }
}

template <int KIND>
__device__ __forceinline__ float update_one(const OptArgs& a, float lr_t, long i, float g) {
  float s1 = 0.f, s2 = 0.f;
  if (KIND != OPT_SGD) s1 = a.s1[i];
  if (KIND == OPT_ADAM || KIND == OPT_RMSPROP) s2 = a.s2[i];
  const float v = upd<KIND>(a, lr_t, a.p[i], g, s1, s2);
  a.p[i] = v;
  if (KIND != OPT_SGD) a.s1[i] = s1;
  if (KIND == OPT_ADAM || KIND == OPT_RMSPROP) a.s2[i] = s2;
  return v;
}

template <bool G16>
__device__ __forceinline__ float load_grad(const OptArgs& a, long i) {
  return (G16 ? bf2f(a.g16[i]) : a.g[i]) * a.gscale;
}

// the updated values' extra destinations: bf16 copies (w16, the ps reply's w16b) and the fp32 copy pb
__device__ __forceinline__ void store_copies(const f32x4_t& p, bf16* w16, bf16* w16b, float* pb) {
  if (w16 || w16b) {
    const u32x2_t q = {pack_bf16x2(p[0], p[1]), pack_bf16x2(p[2], p[3])};
    if (w16) *reinterpret_cast<u32x2_t*>(w16) = q;
    if (w16b) *reinterpret_cast<u32x2_t*>(w16b) = q;
  }
  if (pb) *reinterpret_cast<f32x4_t*>(pb) = p;
}

template <int KIND, bool G16>
__device__ __forceinline__ void update_vec4(const OptArgs& a, float lr_t, long i, bf16* w16, bf16* w16b, float* pb) {
  f32x4_t g;
  if constexpr (!G16) {
    g = *reinterpret_cast<const f32x4_t*>(a.g + i);
  } else {
    const u32x2_t w = *reinterpret_cast<const u32x2_t*>(a.g16 + i);
    g = f32x4_t{__uint_as_float(w[0] << 16), __uint_as_float(w[0] & 0xffff0000u), __uint_as_float(w[1] << 16),
                __uint_as_float(w[1] & 0xffff0000u)};
  }
  f32x4_t p = *reinterpret_cast<const f32x4_t*>(a.p + i);
  f32x4_t s1 = {0.f, 0.f, 0.f, 0.f}, s2 = {0.f, 0.f, 0.f, 0.f};
  if (KIND != OPT_SGD) s1 = *reinterpret_cast<const f32x4_t*>(a.s1 + i);
  if (KIND == OPT_ADAM || KIND == OPT_RMSPROP) s2 = *reinterpret_cast<const f32x4_t*>(a.s2 + i);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    float x1 = s1[j], x2 = s2[j];
    p[j] = upd<KIND>(a, lr_t, p[j], g[j] * a.gscale, x1, x2);
    s1[j] = x1;
    s2[j] = x2;
  }
  *reinterpret_cast<f32x4_t*>(a.p + i) = p;
  if (KIND != OPT_SGD) *reinterpret_cast<f32x4_t*>(a.s1 + i) = s1;
  if (KIND == OPT_ADAM || KIND == OPT_RMSPROP) *reinterpret_cast<f32x4_t*>(a.s2 + i) = s2;
  store_copies(p, w16, w16b, pb);
}

// U vec4 updates at i, i+1024, ... (one workgroup-wide stride apart): every load is issued
// before the first update, so each thread keeps U x (3-4) 16-B loads in flight
template <int KIND, int U, bool G16>
__device__ __forceinline__ void update_vec4x(const OptArgs& a, float lr_t, long i, bf16* w16, bf16* w16b, float* pb) {
  f32x4_t g[U], p[U], s1[U], s2[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const long k = i + u * 1024;
    if constexpr (!G16) {
      g[u] = *reinterpret_cast<const f32x4_t*>(a.g + k);
    } else {
      const u32x2_t w = *reinterpret_cast<const u32x2_t*>(a.g16 + k);
      g[u] = f32x4_t{__uint_as_float(w[0] << 16), __uint_as_float(w[0] & 0xffff0000u), __uint_as_float(w[1] << 16),
                     __uint_as_float(w[1] & 0xffff0000u)};
    }
    p[u] = *reinterpret_cast<const f32x4_t*>(a.p + k);
    s1[u] = s2[u] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    if (KIND != OPT_SGD) s1[u] = *reinterpret_cast<const f32x4_t*>(a.s1 + k);
    if (KIND == OPT_ADAM || KIND == OPT_RMSPROP) s2[u] = *reinterpret_cast<const f32x4_t*>(a.s2 + k);
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const long k = i + u * 1024;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float x1 = s1[u][j], x2 = s2[u][j];
      p[u][j] = upd<KIND>(a, lr_t, p[u][j], g[u][j] * a.gscale, x1, x2);
      s1[u][j] = x1;
      s2[u][j] = x2;
    }
    *reinterpret_cast<f32x4_t*>(a.p + k) = p[u];
    if (KIND != OPT_SGD) *reinterpret_cast<f32x4_t*>(a.s1 + k) = s1[u];
    if (KIND == OPT_ADAM || KIND == OPT_RMSPROP) *reinterpret_cast<f32x4_t*>(a.s2 + k) = s2[u];
    store_copies(p[u], w16 ? w16 + u * 1024 : nullptr, w16b ? w16b + u * 1024 : nullptr, pb ? pb + u * 1024 : nullptr);
  }
}

// One optimizer's share of a launch: workgroups bid = 0..nblk-1 of the grid (the whole grid for a
// plain launch, a contiguous range of it for a grouped one).
template <int KIND, bool G16>
__device__ __forceinline__ void apply_items(const OptArgs& a, int bid, int nblk, bf16 (&tile)[64][66]) {
  float lr_t = a.lr;
  if (KIND == OPT_ADAM) lr_t = tf1_adam_lr(a.lr, a.beta_pow);
  bool waited = false;
  for (int wi = bid; wi < a.nwork; wi += nblk) {
    const OptWork w = a.work[wi];
    const OptSeg sg = a.segs[w.seg];
    if (a.wait_done && !waited && w.seg < 32 && ((a.wait_segs >> w.seg) & 1u)) {
      // the producer (another stream, no graph edge) signals through *wait_done; poll with a bounded
      // wall-clock wait (a producer that never ran: proceed rather than hang the device)
      if (threadIdx.x == 0) {
        const int target = __hip_atomic_load(a.wait_seen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
        const unsigned long long t0 = wall_clock64();
        while (__hip_atomic_load(a.wait_done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target &&
               wall_clock64() - t0 < 200000000ull)  // 2 s at 100 MHz
          __builtin_amdgcn_s_sleep(2);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      }
      __syncthreads();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      waited = true;
    }
    if (w.kind == 0) {
      const long base = sg.off + w.start;
      const long n4 = ((base & 3) == 0) ? (w.count / 4) * 4 : 0;  // segments are 64-aligned; chunks 8192
      long j = threadIdx.x * 4;
      auto at16 = [&](bf16* q, long jj) { return q ? q + w.start + jj : nullptr; };
      auto at32 = [&](float* q, long jj) { return q ? q + w.start + jj : nullptr; };
      for (; j + 3 * 1024 < n4; j += 4 * 1024)  // 4 independent vec4 updates in flight per thread
        update_vec4x<KIND, 4, G16>(a, lr_t, base + j, at16(sg.w16, j), at16(sg.w16b, j), at32(sg.pb, j));
      for (; j < n4; j += 256 * 4)
        update_vec4<KIND, G16>(a, lr_t, base + j, at16(sg.w16, j), at16(sg.w16b, j), at32(sg.pb, j));
      for (long j = n4 + threadIdx.x; j < w.count; j += 256) {
        const long li = w.start + j, i = sg.off + li;
        const float v = update_one<KIND>(a, lr_t, i, load_grad<G16>(a, i));
        if (sg.w16) sg.w16[li] = f2bf(v);
        if (sg.w16b) sg.w16b[li] = f2bf(v);
        if (sg.pb) sg.pb[li] = v;
      }
    } else {
      // 64x64 tile of tap t: rows r0.., cols c0.. of the [R][C] slice; transposed copy via LDS
      // the 16 elements of a thread are loaded together before any update (the update's stores may
      // alias later loads, so a per-element loop ran 16 dependent HBM round trips per workgroup)
      const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
      const int c = w.c0 + tx;
      float gv[16], pv[16], s1v[16], s2v[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const int r = w.r0 + ty + 4 * u;
        // out-of-tile lanes load the segment's first element (never stored): no branches here
        const bool ok = r < sg.R && c < sg.C;
        const long i = sg.off + (ok ? ((long)r * sg.T + w.t) * sg.C + c : 0);
        gv[u] = load_grad<G16>(a, i);
        pv[u] = a.p[i];
        s1v[u] = KIND != OPT_SGD ? a.s1[i] : 0.f;
        s2v[u] = (KIND == OPT_ADAM || KIND == OPT_RMSPROP) ? a.s2[i] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const int rr = ty + 4 * u, r = w.r0 + rr;
        if (r < sg.R && c < sg.C) {
          const long li = ((long)r * sg.T + w.t) * sg.C + c, i = sg.off + li;
          float x1 = s1v[u], x2 = s2v[u];
          const float v = upd<KIND>(a, lr_t, pv[u], gv[u], x1, x2);
          a.p[i] = v;
          if (KIND != OPT_SGD) a.s1[i] = x1;
          if (KIND == OPT_ADAM || KIND == OPT_RMSPROP) a.s2[i] = x2;
          const bf16 b = f2bf(v);
          if (sg.w16) sg.w16[li] = b;
          if (sg.w16b) sg.w16b[li] = b;
          if (sg.pb) sg.pb[li] = v;
          tile[rr][tx] = b;
        }
      }
      __syncthreads();
      for (int cc = ty; cc < 64; cc += 4) {
        const int c = w.c0 + cc, r = w.r0 + tx;
        if (r < sg.R && c < sg.C) {
          const long ti = ((long)c * sg.T + w.t) * sg.R + r;
          if (sg.wt16) sg.wt16[ti] = tile[tx][cc];
          if (sg.wt16b) sg.wt16b[ti] = tile[tx][cc];
        }
      }
      __syncthreads();
    }
  }
}

// the ps reply words (ps_link.h PsWord: REP_GS 9, REP_VER 10, REP_STALE 11, REP_SEQ 8 last) into
// the worker's slot of the host-mapped shared page: system-scope relaxed stores (they go to the
// page, no cache holds them), the sequence number only after the others have completed - no
// release fence: an L2 write-back here would wait for every dirty line the apply just wrote
__device__ __forceinline__ void publish_reply(const OptArgs& a) {
  uint64_t* slot = a.rep_slot;
  const uint64_t gsv = a.rep_gs ? (uint64_t)(int64_t)__hip_atomic_load(const_cast<int32_t*>(a.rep_gs), __ATOMIC_RELAXED,
                                                                         __HIP_MEMORY_SCOPE_AGENT)
                                : (uint64_t)(int64_t)-1;
  __hip_atomic_store(slot + 9, gsv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(slot + 10, a.rep_ver, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(slot + 11, (uint64_t)a.rep_stale, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __hip_atomic_store(slot + 8, a.rep_seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

template <int KIND>
__device__ __forceinline__ void apply_body(const OptArgs& a, int bid, int nblk, bf16 (&tile)[64][66]) {
  if (a.g) apply_items<KIND, false>(a, bid, nblk, tile);
  else apply_items<KIND, true>(a, bid, nblk, tile);
  // last workgroup: advance the non-slot scalars.  Every thread read them at its start and
  // used the value; after the barrier one lane takes a ticket (relaxed agent atomics - nothing
  // is handed between workgroups, so no fences) and the last arriver updates them.
  // A folded ps reply is handed over: every wave's stores (the reply buffer copies, uncached
  // memory) have completed before its workgroup takes the ticket, so the last arriver's reply
  // words follow every value the worker will read.
  if (a.rep_slot) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t prev = __hip_atomic_fetch_add(a.done_counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (prev == (uint32_t)nblk - 1 && !a.skip_advance) {
      if (KIND == OPT_ADAM) {
        a.beta_pow[0] *= a.beta1;
        a.beta_pow[1] *= a.beta2;
      }
      if (a.global_step && a.gs_inc) atomicAdd(a.global_step, a.gs_inc);
    }
    if (prev == (uint32_t)nblk - 1 && a.wait_seen)
      __hip_atomic_fetch_add(a.wait_seen, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (prev == (uint32_t)nblk - 1 && a.rep_slot) publish_reply(a);
    if (prev == (uint32_t)nblk - 1) __hip_atomic_store(a.done_counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

template <int KIND>
__global__ __launch_bounds__(256) void apply_gradients_kernel(OptArgs a) {
  __shared__ __attribute__((aligned(16))) bf16 tile[64][66];
  apply_body<KIND>(a, blockIdx.x, gridDim.x, tile);
}

// Several optimizers of one kind in ONE launch (the GAN's two Adams over disjoint var lists):
// workgroup ranges [first[i], first[i + 1]) run optimizer i; each keeps its own done counter,
// beta powers and global-step increment, exactly as separate launches would.
template <int KIND>
__global__ __launch_bounds__(256) void apply_gradients_group_kernel(OptGroup g) {
  __shared__ __attribute__((aligned(16))) bf16 tile[64][66];
  int i = 0;
  while (i + 1 < g.n && (int)blockIdx.x >= g.first[i + 1]) ++i;
  apply_body<KIND>(g.o[i], blockIdx.x - g.first[i], g.first[i + 1] - g.first[i], tile);
}

__device__ __forceinline__ void advance_one(const OptArgs& a) {
  if (a.kind == OPT_ADAM && a.beta_pow) {
    a.beta_pow[0] *= a.beta1;
    a.beta_pow[1] *= a.beta2;
  }
  if (a.global_step && a.gs_inc) atomicAdd(a.global_step, a.gs_inc);
}

__global__ void opt_advance_kernel(OptArgs a) {
  if (threadIdx.x != 0) return;
  advance_one(a);
}

struct OptAdvanceSet {
  OptArgs o[OPT_GROUP_MAX];
  int n;
};
__global__ void opt_advance_reply_kernel(OptAdvanceSet g) {
  if (threadIdx.x != 0) return;
  for (int i = 0; i < g.n; ++i) advance_one(g.o[i]);
  if (g.o[g.n - 1].rep_slot) publish_reply(g.o[g.n - 1]);
}

__global__ void epoch_signal_kernel(int* ctr) {
  if (threadIdx.x == 0) __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}
void launch_epoch_signal(int* ctr, hipStream_t s) { hipLaunchKernelGGL(epoch_signal_kernel, dim3(1), dim3(64), 0, s, ctr); }

static int apply_blocks(const OptArgs& a) {
  int blocks = a.nwork < 2048 ? a.nwork : 2048;
  return blocks < 1 ? 1 : blocks;
}

void launch_apply_gradients_group(const OptArgs* o, int n, hipStream_t s) {
  if (n < 1 || n > OPT_GROUP_MAX) throw std::runtime_error("apply_gradients_group: 1..4 optimizers");
  OptGroup g{};
  g.n = n;
  g.first[0] = 0;
  for (int i = 0; i < n; ++i) {
    if (o[i].kind != o[0].kind) throw std::runtime_error("apply_gradients_group: one optimizer kind per launch");
    g.o[i] = o[i];
    g.first[i + 1] = g.first[i] + apply_blocks(o[i]);
  }
  const dim3 grid(g.first[n]);
  switch (o[0].kind) {
    case OPT_SGD: hipLaunchKernelGGL(apply_gradients_group_kernel<OPT_SGD>, grid, dim3(256), 0, s, g); break;
    case OPT_MOMENTUM: hipLaunchKernelGGL(apply_gradients_group_kernel<OPT_MOMENTUM>, grid, dim3(256), 0, s, g); break;
    case OPT_ADAM: hipLaunchKernelGGL(apply_gradients_group_kernel<OPT_ADAM>, grid, dim3(256), 0, s, g); break;
    default: hipLaunchKernelGGL(apply_gradients_group_kernel<OPT_RMSPROP>, grid, dim3(256), 0, s, g); break;
  }
}

void launch_opt_advance(const OptArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(opt_advance_kernel, dim3(1), dim3(64), 0, s, a);
}

void launch_opt_advance_reply(const OptArgs* a, int n, hipStream_t s) {
  if (n < 1 || n > OPT_GROUP_MAX) throw std::runtime_error("opt_advance_reply: 1..4 optimizers");
  OptAdvanceSet g{};
  for (int i = 0; i < n; ++i) g.o[i] = a[i];
  g.n = n;
  hipLaunchKernelGGL(opt_advance_reply_kernel, dim3(1), dim3(64), 0, s, g);
}

void launch_apply_gradients(const OptArgs& a, hipStream_t s) {
  const int blocks = apply_blocks(a);
  switch (a.kind) {
    case OPT_SGD: hipLaunchKernelGGL(apply_gradients_kernel<OPT_SGD>, dim3(blocks), dim3(256), 0, s, a); break;
    case OPT_MOMENTUM:
      hipLaunchKernelGGL(apply_gradients_kernel<OPT_MOMENTUM>, dim3(blocks), dim3(256), 0, s, a);
      break;
    case OPT_ADAM: hipLaunchKernelGGL(apply_gradients_kernel<OPT_ADAM>, dim3(blocks), dim3(256), 0, s, a); break;
    default: hipLaunchKernelGGL(apply_gradients_kernel<OPT_RMSPROP>, dim3(blocks), dim3(256), 0, s, a); break;
  }
}

}  // namespace dtfe
