// Parameter-server data-plane kernels (see ps_link.h).
#include "ps_link.h"

namespace dtfe {

namespace {

__device__ __forceinline__ void st_sys(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint64_t ld_sys(const uint64_t* p) {
  return __hip_atomic_load(const_cast<uint64_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void drain_stores() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// Hand-off discipline (no release fences; one acquire in ps_wait_kernel): mailboxes and reply buffers are uncached
// device memory, so a store is in memory once it has completed; every copy kernel drains its
// stores before it ends (the next kernel of the stream starts after it), and the handshake
// words are system-scope relaxed stores to the host-mapped page, the sequence number issued
// only after the other words have completed.  A system-scope release fence would instead write
// back every dirty line of the XCD's L2 - tens of microseconds after an apply or a backward
// (profiles/r4_ps_1p1w_timeline.txt: ps_reply 41-47 us, ps_request 3-4 us).

__device__ __forceinline__ void cvt8(const void* src, int smode_bf16, long i, float (&v)[8]) {
  if (smode_bf16) {
    const u32x4_t w = *reinterpret_cast<const u32x4_t*>(reinterpret_cast<const bf16*>(src) + i);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      v[2 * k] = __uint_as_float(w[k] << 16);
      v[2 * k + 1] = __uint_as_float(w[k] & 0xffff0000u);
    }
  } else {
    const f32x4_t* q = reinterpret_cast<const f32x4_t*>(reinterpret_cast<const float*>(src) + i);
    const f32x4_t lo = q[0], hi = q[1];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      v[k] = lo[k];
      v[4 + k] = hi[k];
    }
  }
}

// 8 elements at i: vector path (every pointer of these plans is 16-B aligned at element 0)
__device__ __forceinline__ void copy8(const PsSeg& s, long i) {
  if (s.mode == 2) {  // bf16 -> bf16: one 16 B move
    *reinterpret_cast<u32x4_t*>(reinterpret_cast<bf16*>(s.dst) + i) =
        *reinterpret_cast<const u32x4_t*>(reinterpret_cast<const bf16*>(s.src) + i);
    return;
  }
  if (s.mode == 0) {
    const f32x4_t* q = reinterpret_cast<const f32x4_t*>(reinterpret_cast<const float*>(s.src) + i);
    f32x4_t* d = reinterpret_cast<f32x4_t*>(reinterpret_cast<float*>(s.dst) + i);
    const f32x4_t a = q[0], b = q[1];
    d[0] = a;
    d[1] = b;
    return;
  }
  float v[8];
  cvt8(s.src, s.mode == 3 || s.mode == 5, i, v);
  if (s.mode == 1) {
    *reinterpret_cast<u32x4_t*>(reinterpret_cast<bf16*>(s.dst) + i) =
        u32x4_t{pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]), pack_bf16x2(v[4], v[5]), pack_bf16x2(v[6], v[7])};
    return;
  }
  f32x4_t* d = reinterpret_cast<f32x4_t*>(reinterpret_cast<float*>(s.dst) + i);
  if (s.mode == 3) {
    d[0] = f32x4_t{v[0], v[1], v[2], v[3]};
    d[1] = f32x4_t{v[4], v[5], v[6], v[7]};
  } else {  // 4 / 5: accumulate
    const f32x4_t a = d[0], b = d[1];
    d[0] = a + f32x4_t{v[0], v[1], v[2], v[3]};
    d[1] = b + f32x4_t{v[4], v[5], v[6], v[7]};
  }
}

__device__ __forceinline__ void copy1(const PsSeg& s, long i) {
  const bool sb = s.mode == 2 || s.mode == 3 || s.mode == 5;
  const float v = sb ? bf2f(reinterpret_cast<const bf16*>(s.src)[i]) : reinterpret_cast<const float*>(s.src)[i];
  switch (s.mode) {
    case 1:
    case 2: reinterpret_cast<bf16*>(s.dst)[i] = f2bf(v); break;
    case 4:
    case 5: reinterpret_cast<float*>(s.dst)[i] += v; break;
    default: reinterpret_cast<float*>(s.dst)[i] = v; break;
  }
}

__global__ __launch_bounds__(256) void ps_copy_kernel(const PsSeg* __restrict__ segs, const PsWork* __restrict__ work,
                                                      int nwork) {
  for (int wi = blockIdx.x; wi < nwork; wi += gridDim.x) {
    const PsWork w = work[wi];
    const PsSeg s = segs[w.seg];
    const long n8 = (w.count / 8) * 8;
    for (long j = (long)threadIdx.x * 8; j < n8; j += 256 * 8) copy8(s, w.start + j);
    for (long j = n8 + threadIdx.x; j < w.count; j += 256) copy1(s, w.start + j);
  }
  drain_stores();  // a push / reply is complete in (uncached) memory when the kernel ends
}

__global__ void ps_request_kernel(uint64_t* slot, int64_t* ctr, const int64_t* ver, int kind, int bump) {
  if (threadIdx.x != 0) return;
  // one exchange = one request number for every shard: only the first shard's request advances
  // the counter (the others follow it on the same stream and reuse the value)
  const int64_t c = *ctr + bump;
  if (bump) *ctr = c;
  // every preceding kernel of this stream (the push copies) has completed and drained its stores
  st_sys(slot + PS_REQ_KIND, (uint64_t)kind);
  st_sys(slot + PS_REQ_TAG, ver ? (uint64_t)*ver : 0ull);
  drain_stores();
  st_sys(slot + PS_REQ_SEQ, (uint64_t)c);
}

__global__ void ps_bucket_kernel(uint64_t* slot, const int64_t* ctr, int b, long lo, long hi) {
  if (threadIdx.x != 0) return;
  // the bucket's push copies (earlier on this stream) have completed: publish its range
  st_sys(slot + PS_BKT_BASE + 3 * b + 1, (uint64_t)lo);
  st_sys(slot + PS_BKT_BASE + 3 * b + 2, (uint64_t)hi);
  drain_stores();
  st_sys(slot + PS_BKT_BASE + 3 * b, (uint64_t)(*ctr + 1));
}

__global__ void ps_wait_kernel(PsWaitArgs a) {
  if (threadIdx.x != 0) return;
  const uint64_t target = (uint64_t)*a.ctr;
  const unsigned long long t0 = wall_clock64();
  for (int k = 0; k < a.nslots; ++k) {
    while (ld_sys(a.slot[k] + PS_REP_SEQ) < target) {
      if (wall_clock64() - t0 > a.timeout_ticks) {
        atomicExch(a.err, 1);
        return;
      }
      __builtin_amdgcn_s_sleep(4);
    }
  }
  // system-scope acquire: one cache invalidate on the waiting side.  The reply buffers are allocated
  // uncached by their exporter, but the pull that follows may read them through a hipIpc import on
  // ANOTHER GPU, whose mapping attributes this code does not control - stale lines of an earlier
  // reply in that GPU's L2 must not be served to the pull (the release side stays fence-free: its
  // stores are drained to uncached memory, see the note above)
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  if (a.gs_out && a.gs_slot >= 0) *a.gs_out = (int32_t)(int64_t)ld_sys(a.slot[a.gs_slot] + PS_REP_GS);
  if (a.ver_out)  // per shard: each shard's version is the staleness tag of that shard's next request
    for (int k = 0; k < a.nslots; ++k) a.ver_out[k] = (int64_t)ld_sys(a.slot[k] + PS_REP_VER);
}

__global__ void ps_reply_kernel(uint64_t* slot, const int32_t* gs, uint64_t seq, uint64_t ver, int stale) {
  if (threadIdx.x != 0) return;
  // the reply snapshot (earlier on this stream) has completed and drained its stores
  st_sys(slot + PS_REP_GS, gs ? (uint64_t)(int64_t)*gs : (uint64_t)(int64_t)-1);
  st_sys(slot + PS_REP_VER, ver);
  st_sys(slot + PS_REP_STALE, (uint64_t)stale);
  drain_stores();
  st_sys(slot + PS_REP_SEQ, seq);
}

}  // namespace

void launch_ps_copy(const PsSeg* segs, const PsWork* work, int nwork, hipStream_t s) {
  if (nwork <= 0) return;
  const int blocks = nwork < 2048 ? nwork : 2048;
  hipLaunchKernelGGL(ps_copy_kernel, dim3(blocks), dim3(256), 0, s, segs, work, nwork);
}

void launch_ps_request(uint64_t* slot, int64_t* ctr, const int64_t* ver, int kind, int bump, hipStream_t s) {
  hipLaunchKernelGGL(ps_request_kernel, dim3(1), dim3(64), 0, s, slot, ctr, ver, kind, bump);
}

void launch_ps_bucket(uint64_t* slot, const int64_t* ctr, int b, long lo, long hi, hipStream_t s) {
  hipLaunchKernelGGL(ps_bucket_kernel, dim3(1), dim3(64), 0, s, slot, ctr, b, lo, hi);
}

void launch_ps_wait(const PsWaitArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(ps_wait_kernel, dim3(1), dim3(64), 0, s, a);
}

void launch_ps_reply(uint64_t* slot, const int32_t* gs, uint64_t seq, uint64_t ver, int stale, hipStream_t s) {
  hipLaunchKernelGGL(ps_reply_kernel, dim3(1), dim3(64), 0, s, slot, gs, seq, ver, stale);
}

}  // namespace dtfe
