// Cost of cross-workgroup reductions on one MI355X: per-launch time of a grid whose workgroups
// each end with (a) nothing, (b) one relaxed agent-scope ticket atomic on a shared counter,
// (c) 2C float atomics onto a [2][C] statistics vector (bn_stats' reduction), C = 16 / 64.
//   hipcc -O3 --offload-arch=gfx950 bench/atomic_contention.hip -o /tmp/atomic_contention
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void k_none(float* out) {
  __shared__ float s[256];
  s[threadIdx.x] = threadIdx.x;
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = s[255];
}

__global__ void k_ticket(float* out, unsigned* ctr) {
  __shared__ float s[256];
  s[threadIdx.x] = threadIdx.x;
  __syncthreads();
  if (threadIdx.x == 0) {
    out[blockIdx.x] = s[255];
    unsigned t = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (t == gridDim.x - 1) __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

__global__ void k_stats(float* out, float* stats, int n2c) {
  __shared__ float s[256];
  s[threadIdx.x] = threadIdx.x;
  __syncthreads();
  if (threadIdx.x < n2c) atomicAdd(stats + threadIdx.x, s[threadIdx.x] * 1e-9f);
  if (threadIdx.x == 0) out[blockIdx.x] = s[255];
}

int main() {
  float *out, *stats;
  unsigned* ctr;
  (void)hipMalloc(&out, 4096 * sizeof(float));
  (void)hipMalloc(&stats, 256 * sizeof(float));
  (void)hipMalloc(&ctr, 64);
  (void)hipMemset(ctr, 0, 64);
  (void)hipMemset(stats, 0, 256 * sizeof(float));
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int N = 400;
  printf("%-22s %6s %10s\n", "kernel", "grid", "us/launch");
  for (int grid : {64, 128, 256, 512}) {
    for (int kind = 0; kind < 4; ++kind) {
      auto launch = [&]() {
        if (kind == 0) hipLaunchKernelGGL(k_none, dim3(grid), dim3(256), 0, 0, out);
        if (kind == 1) hipLaunchKernelGGL(k_ticket, dim3(grid), dim3(256), 0, 0, out, ctr);
        if (kind == 2) hipLaunchKernelGGL(k_stats, dim3(grid), dim3(256), 0, 0, out, stats, 32);
        if (kind == 3) hipLaunchKernelGGL(k_stats, dim3(grid), dim3(256), 0, 0, out, stats, 128);
      };
      for (int i = 0; i < 20; ++i) launch();
      (void)hipDeviceSynchronize();
      (void)hipEventRecord(e0, 0);
      for (int i = 0; i < N; ++i) launch();
      (void)hipEventRecord(e1, 0);
      (void)hipEventSynchronize(e1);
      float ms = 0;
      (void)hipEventElapsedTime(&ms, e0, e1);
      static const char* names[] = {"none", "ticket (1 addr)", "stats 2C=32 atomics", "stats 2C=128 atomics"};
      printf("%-22s %6d %10.2f\n", names[kind], grid, ms * 1000.0f / N);
    }
  }
  return 0;
}
