// Two-shot all-reduce over hipIpc-mapped peer memory.
//
// Every rank owns one exchange buffer allocated UNCACHED (hipDeviceMallocUncached)
// and mapped into every other rank's address space with hipIpcOpenMemHandle, so
// a plain load of a peer's buffer is a direct xGMI read and nothing a peer wrote
// can hide in this GPU's L1/L2.  One launch does the whole collective:
//
//   A  stage:  each workgroup copies its slice of every segment of the input into
//              this rank's staging buffer (parity = call number & 1)
//      barrier 0 (per workgroup, all ranks: "my slice is staged")
//   B  reduce: workgroup b sums ITS slice of segment `rank` over all W staging
//              buffers (W-1 xGMI reads in flight per thread, fp32 accumulation)
//              and writes the result to the output and back into its staging slice
//      barrier 1 ("my reduced slice is published")
//   C  gather: copy every other segment's reduced slice from its owner
//
// Per rank that is 2*(W-1)/W of the bytes read over the fabric, spread over all
// W-1 point-to-point links at once (each link carries 2/W of the buffer) - the
// reduce-scatter + all-gather of a ring without its 2(W-1) dependent steps.
// Barriers are per workgroup (block b only ever touches slice b of each segment)
// with monotonically increasing epoch values, so no flag is ever reset; the two
// staging parities keep call s+1's staging writes away from readers still in
// call s's gather.  Every wait has a wall-clock timeout: a missing peer sets
// *err and the kernel exits instead of hanging the GPU.
#include "ipc_allreduce.h"

#include "common.h"

namespace dtfe {

namespace {

__device__ __forceinline__ uint32_t* ipc_flag(char* base, int ph, int b, int src) {
  return reinterpret_cast<uint32_t*>(base) + ((long)ph * IPC_MAXB + b) * IPC_MAXW + src;
}

// Returns false (block-uniformly) when a peer did not arrive before the timeout.
__device__ __forceinline__ bool ipc_barrier(const IpcAllReduceArgs& a, int ph, uint32_t ep, int* s_ok) {
  // this wave's staging / output stores are performed (uncached memory: at the memory side)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const int t = threadIdx.x;
  if (t < a.world) {
    __hip_atomic_store(ipc_flag(a.base[t], ph, blockIdx.x, a.rank), ep, __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_SYSTEM);
    uint32_t* f = ipc_flag(a.base[a.rank], ph, blockIdx.x, t);
    const unsigned long long t0 = wall_clock64();
    while ((int)(__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) - ep) < 0) {
      if (wall_clock64() - t0 > a.timeout) {
        atomicExch(a.err, 1);
        *s_ok = 0;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __syncthreads();
  return *s_ok != 0;
}

// The last block of a launch to finish advances the launch counter (every block read it at its
// start; the next launch on this stream only begins after this one completed).
__device__ __forceinline__ void ipc_block_done(const IpcAllReduceArgs& a) {
  if (threadIdx.x == 0 && atomicAdd(a.calls + 1, 1u) == (uint32_t)a.blocks - 1) {
    a.calls[1] = 0;
    atomicAdd(a.calls, 1u);
  }
}

template <typename T> struct Vec16;
template <> struct Vec16<bf16> {
  static constexpr int N = 8;
  __device__ static void add(float (&acc)[8], uint4 v) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      acc[2 * k] += __uint_as_float(w[k] << 16);
      acc[2 * k + 1] += __uint_as_float(w[k] & 0xffff0000u);
    }
  }
  __device__ static uint4 pack(const float (&acc)[8]) {
    return uint4{pack_bf16x2(acc[0], acc[1]), pack_bf16x2(acc[2], acc[3]), pack_bf16x2(acc[4], acc[5]),
                 pack_bf16x2(acc[6], acc[7])};
  }
  __device__ static float ld(const bf16* p) { return bf2f(*p); }
  __device__ static void st(bf16* p, float v) { *p = f2bf(v); }
};
template <> struct Vec16<float> {
  static constexpr int N = 4;
  __device__ static void add(float (&acc)[4], uint4 v) {
    acc[0] += __uint_as_float(v.x);
    acc[1] += __uint_as_float(v.y);
    acc[2] += __uint_as_float(v.z);
    acc[3] += __uint_as_float(v.w);
  }
  __device__ static uint4 pack(const float (&acc)[4]) {
    return uint4{__float_as_uint(acc[0]), __float_as_uint(acc[1]), __float_as_uint(acc[2]), __float_as_uint(acc[3])};
  }
  __device__ static float ld(const float* p) { return *p; }
  __device__ static void st(float* p, float v) { *p = v; }
};

template <typename T, int W>
__global__ __launch_bounds__(IPC_THREADS) void ipc_allreduce_kernel(IpcAllReduceArgs a) {
  using V = Vec16<T>;
  __shared__ uint32_t s_ep, s_par;
  __shared__ int s_ok;
  const int tid = threadIdx.x, b = blockIdx.x, r = a.rank;
  if (tid == 0) {
    s_ep = a.epoch[b] + 1;
    s_par = a.calls[0] & 1u;
    s_ok = 1;
  }
  __syncthreads();
  const uint32_t ep = s_ep;
  // The staging parity flips once per LAUNCH, identically for every block and rank.  (A
  // per-block parity would not do: launches of different sizes run different block counts,
  // so block b's slice and its epoch differ between calls, and a fast rank's next-call
  // staging could land on the parity a slow peer is still gathering from.)
  const long off = IPC_DATA_OFF + (long)s_par * a.cap;
  // 16-B body plus up to 2*(V::N-1) scalar elements (the unaligned head before the first
  // 16-B boundary and the tail) that block 0 of every rank reduces on its own
  T* const x = reinterpret_cast<T*>(a.buf);
  const int hd = (int)(((16 - (reinterpret_cast<uintptr_t>(x) & 15)) & 15) / sizeof(T));
  const long nb = a.n > hd ? a.n - hd : 0;
  const int head = (int)(a.n < hd ? a.n : hd);
  const long nvec = nb / V::N;
  const int ns = head + (int)(nb - nvec * V::N);
  const long seg = (nvec + W - 1) / W;
  const long step = (long)a.blocks * IPC_THREADS;
  const long i0 = (long)b * IPC_THREADS + tid;
  uint4* io = reinterpret_cast<uint4*>(x + head);
  uint4* mine = reinterpret_cast<uint4*>(a.base[r] + off);
  T* sx = nullptr;  // this thread's scalar element (block 0, tid < ns)
  if (b == 0 && tid < ns) sx = tid < head ? x + tid : x + head + nvec * V::N + (tid - head);

  // A: stage this block's slice of every segment
#pragma unroll
  for (int p = 0; p < W; ++p) {
    const long hi = min(nvec, (p + 1) * seg);
    for (long i = p * seg + i0; i < hi; i += step) mine[i] = io[i];
  }
  if (sx) reinterpret_cast<T*>(mine + nvec)[tid] = *sx;
  if (!ipc_barrier(a, 0, ep, &s_ok)) {
    ipc_block_done(a);
    return;
  }

  // B: reduce this block's slice of segment r over every rank's staging buffer
  {
    const long hi = min(nvec, (r + 1) * seg);
    for (long i = r * seg + i0; i < hi; i += step) {
      uint4 v[W];
#pragma unroll
      for (int q = 0; q < W; ++q) v[q] = reinterpret_cast<const uint4*>(a.base[q] + off)[i];
      float acc[V::N];
#pragma unroll
      for (int e = 0; e < V::N; ++e) acc[e] = 0.f;
#pragma unroll
      for (int q = 0; q < W; ++q) V::add(acc, v[q]);
      const uint4 o = V::pack(acc);
      mine[i] = o;
      io[i] = o;
    }
    if (sx) {
      float s = 0.f;
#pragma unroll
      for (int q = 0; q < W; ++q)
        s += V::ld(reinterpret_cast<const T*>(reinterpret_cast<const uint4*>(a.base[q] + off) + nvec) + tid);
      V::st(sx, s);
    }
  }
  if (!ipc_barrier(a, 1, ep, &s_ok)) {
    ipc_block_done(a);
    return;
  }

  // C: gather the other ranks' reduced segments
#pragma unroll
  for (int p = 0; p < W; ++p) {
    if (p == r) continue;
    const uint4* src = reinterpret_cast<const uint4*>(a.base[p] + off);
    const long hi = min(nvec, (p + 1) * seg);
    for (long i = p * seg + i0; i < hi; i += step) io[i] = src[i];
  }
  if (tid == 0) a.epoch[b] = ep;
  ipc_block_done(a);
}

template <typename T>
void launch_t(const IpcAllReduceArgs& a, hipStream_t s) {
  const dim3 g(a.blocks), blk(IPC_THREADS);
  switch (a.world) {
    case 1: hipLaunchKernelGGL((ipc_allreduce_kernel<T, 1>), g, blk, 0, s, a); break;
    case 2: hipLaunchKernelGGL((ipc_allreduce_kernel<T, 2>), g, blk, 0, s, a); break;
    case 3: hipLaunchKernelGGL((ipc_allreduce_kernel<T, 3>), g, blk, 0, s, a); break;
    case 4: hipLaunchKernelGGL((ipc_allreduce_kernel<T, 4>), g, blk, 0, s, a); break;
    case 5: hipLaunchKernelGGL((ipc_allreduce_kernel<T, 5>), g, blk, 0, s, a); break;
    case 6: hipLaunchKernelGGL((ipc_allreduce_kernel<T, 6>), g, blk, 0, s, a); break;
    case 7: hipLaunchKernelGGL((ipc_allreduce_kernel<T, 7>), g, blk, 0, s, a); break;
    case 8: hipLaunchKernelGGL((ipc_allreduce_kernel<T, 8>), g, blk, 0, s, a); break;
    default: break;
  }
}

}  // namespace

void launch_ipc_allreduce(const IpcAllReduceArgs& a, int dtype, hipStream_t s) {
  if (dtype == 0) launch_t<bf16>(a, s);
  else launch_t<float>(a, s);
}

}  // namespace dtfe
