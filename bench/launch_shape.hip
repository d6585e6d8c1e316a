// In-graph cost of an (almost) empty launch by shape: grid x threads x dynamic LDS, 100 launches
// captured in one hipGraph, replayed 20x.  How much of a short persistent kernel (ResNet-20's
// whole-image convs: 256 x 1024 threads, ~100 KB LDS) is launch shape rather than work.
//   hipcc -O3 --offload-arch=gfx950 bench/launch_shape.hip -o /tmp/launch_shape
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void k_empty(float* out) {
  extern __shared__ float lds[];
  if (threadIdx.x == 0) lds[0] = 1.f;
  __syncthreads();
  if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = lds[0];
}

int main() {
  float* out;
  (void)hipMalloc(&out, 64);
  (void)hipFuncSetAttribute((const void*)k_empty, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  hipStream_t s;
  (void)hipStreamCreate(&s);
  printf("%6s %8s %8s %10s\n", "grid", "threads", "LDS KB", "us/launch");
  for (int grid : {1, 256, 512}) {
    for (int thr : {256, 512, 1024}) {
      for (int kb : {0, 64, 128}) {
        hipGraph_t g;
        hipGraphExec_t ge;
        (void)hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
        for (int i = 0; i < 100; ++i) hipLaunchKernelGGL(k_empty, dim3(grid), dim3(thr), kb * 1024, s, out);
        (void)hipStreamEndCapture(s, &g);
        (void)hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
        for (int w = 0; w < 3; ++w) (void)hipGraphLaunch(ge, s);
        (void)hipStreamSynchronize(s);
        hipEvent_t e0, e1;
        (void)hipEventCreate(&e0);
        (void)hipEventCreate(&e1);
        (void)hipEventRecord(e0, s);
        for (int r = 0; r < 20; ++r) (void)hipGraphLaunch(ge, s);
        (void)hipEventRecord(e1, s);
        (void)hipEventSynchronize(e1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        printf("%6d %8d %8d %10.2f\n", grid, thr, kb, ms * 1000.f / 2000.f);
        (void)hipGraphExecDestroy(ge);
        (void)hipGraphDestroy(g);
      }
    }
  }
  return 0;
}
