// global_load_lds streaming probe (diagnostic, not part of the library): how many bytes per clock
// per CU the LDS-DMA path moves for the MNIST-CNN fc1 access shape as a function of the contiguous
// segment length per row.  Every workgroup streams a 64-row block of a [rows][ld] bf16 matrix
// (L2 / Infinity-Cache resident, like fc1's operands) in k-tiles of SEG bytes per row, 3 stages in
// flight (counted vmcnt + raw s_barrier, the gemm_glds.h loop without the MFMAs).
//   hipcc --offload-arch=gfx950 -O3 bench/probe/glds_probe.hip -o bench/probe/glds_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef __attribute__((address_space(3))) void lds_t;

template <int SEG, int STAGES, int THREADS = 256>
__device__ __forceinline__ void stream_body(const unsigned short* src, int ld, int kbytes, int blocks_m,
                                                        int* sink) {
  constexpr int TILE = 64 * SEG;                 // bytes per k-tile (64 rows)
  constexpr int NW = THREADS / 64;
  constexpr int PIECES = TILE / (THREADS * 16);  // 16-B DMA pieces per thread per k-tile
  static_assert(PIECES >= 1, "at least one piece per thread");
  constexpr int CPR = SEG / 16, RPP = 64 / CPR;  // chunks per row, rows per 1 KB piece
  __shared__ __attribute__((aligned(16))) unsigned char lds[STAGES * TILE];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int rb = (blockIdx.x % blocks_m) * 64;
  const unsigned char* base = reinterpret_cast<const unsigned char*>(src) + (long)rb * ld * 2;
  const unsigned char* p[PIECES];
#pragma unroll
  for (int j = 0; j < PIECES; ++j) {
    const int row = (j * NW + w) * RPP + lane / CPR, chunk = lane % CPR;
    p[j] = base + (long)row * ld * 2 + chunk * 16;
  }
  const int nk = kbytes / SEG;
  auto issue = [&](int kt, int s) {
#pragma unroll
    for (int j = 0; j < PIECES; ++j)
      __builtin_amdgcn_global_load_lds(p[j] + (long)kt * SEG, (lds_t*)(lds + s * TILE + (j * NW + w) * 1024), 16, 0, 0);
  };
  for (int s = 0; s < STAGES - 1 && s < nk; ++s) issue(s, s);
  int acc = 0;
  for (int t = 0; t < nk; ++t) {
    if (t + STAGES - 2 < nk) asm volatile("s_waitcnt vmcnt(%0)" ::"n"((STAGES - 2) * PIECES) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (t + STAGES - 1 < nk) issue(t + STAGES - 1, (t + STAGES - 1) % STAGES);
    acc += lds[(t % STAGES) * TILE + threadIdx.x * 4];  // touch the tile
  }
  if (acc == 0x7fffffff) sink[0] = acc;
}


#define PROBE(S, T) \
  __global__ __launch_bounds__(256, 1) void k_##S##_##T(const unsigned short* src, int ld, int kb, int bm, int* sink) { \
    stream_body<S, T>(src, ld, kb, bm, sink); \
  }
PROBE(128, 3)
PROBE(256, 3)
PROBE(512, 3)
PROBE(128, 4)
PROBE(256, 4)
// waves per workgroup: one workgroup of 8 / 16 waves per CU vs several 4-wave workgroups
#define PROBET(S, T, TH) \
  __global__ __launch_bounds__(TH, 1) void k_##S##_##T##_##TH(const unsigned short* src, int ld, int kb, int bm, int* sink) { \
    stream_body<S, T, TH>(src, ld, kb, bm, sink); \
  }
PROBET(128, 3, 512)
PROBET(256, 3, 512)
PROBET(256, 3, 1024)
PROBET(128, 6, 512)

typedef void (*Kern)(const unsigned short*, int, int, int, int*);

double run(Kern k, int SEG, int STAGES, const unsigned short* d, int rows, int ld, int grid, int* sink, int th = 256) {
  const int blocks_m = rows / 64, kbytes = (ld * 2 / SEG) * SEG;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(k, dim3(grid), dim3(th), 0, 0, d, ld, kbytes, blocks_m, sink);
  hipEventRecord(e0);
  const int reps = 20;
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(k, dim3(grid), dim3(th), 0, 0, d, ld, kbytes, blocks_m, sink);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  const double us = ms * 1000.0 / reps;
  const double bytes = (double)grid * 64 * kbytes;
  printf("SEG %4d B  stages %d  threads %4d  grid %4d : %7.1f us  %6.2f TB/s  %5.1f B/clk/CU (2.4 GHz)\n", SEG, STAGES, th, grid, us,
         bytes / us / 1e6, bytes / (us * 1e-6) / 2.4e9 / 256);
  (void)th;
  return us;
}

int main() {
  const int rows = 1024, ld = 3200;  // 6.5 MB, row pitch a multiple of every SEG
  unsigned short* d;
  int* sink;
  hipMalloc(&d, (size_t)rows * ld * 2);
  hipMalloc(&sink, 4);
  hipMemset(d, 1, (size_t)rows * ld * 2);
  // one workgroup per CU with 8 / 16 waves (grid 256), and 2 x 8 waves (grid 512)
  for (int grid : {256, 512}) {
    run(k_128_3_512, 128, 3, d, rows, ld, grid, sink, 512);
    run(k_256_3_512, 256, 3, d, rows, ld, grid, sink, 512);
    run(k_128_6_512, 128, 6, d, rows, ld, grid, sink, 512);
  }
  run(k_256_3_1024, 256, 3, d, rows, ld, 256, sink, 1024);
  for (int grid : {256, 512, 768}) {
    run(k_128_3, 128, 3, d, rows, ld, grid, sink);
    run(k_256_3, 256, 3, d, rows, ld, grid, sink);
    run(k_512_3, 512, 3, d, rows, ld, grid, sink);
    run(k_128_4, 128, 4, d, rows, ld, grid, sink);
    run(k_256_4, 256, 4, d, rows, ld, grid, sink);
  }
  hipFree(d);
  return 0;
}
