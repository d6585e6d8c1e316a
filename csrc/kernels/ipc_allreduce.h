// Two-shot all-reduce over hipIpc-mapped peer buffers.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dtfe {

constexpr int IPC_MAXW = 8;      // ranks (one node: 8 GPUs, 7 xGMI peers each)
constexpr int IPC_MAXB = 128;    // workgroups per launch (each owns a slice of every segment)
constexpr int IPC_THREADS = 512;
// per-rank exchange buffer: [flags: 2 barriers x IPC_MAXB blocks x IPC_MAXW sources u32]
// [pad to IPC_DATA_OFF] [parity 0 staging: cap bytes] [parity 1 staging: cap bytes]
constexpr long IPC_DATA_OFF = 64 * 1024;

struct IpcAllReduceArgs {
  char* base[IPC_MAXW];  // every rank's exchange buffer in THIS process's address space (own included)
  long cap;              // staging bytes per parity
  int rank, world;
  void* buf;             // in/out tensor (in place)
  long n;                // elements
  uint32_t* epoch;       // [IPC_MAXB] per-block call counters (local memory)
  uint32_t* calls;       // [2] {launches completed, blocks finished in the current launch} (local memory)
  int* err;              // set to 1 when a barrier timed out
  unsigned long long timeout;  // wall_clock64 ticks (100 MHz)
  int blocks;
};

// dtype: 0 = bf16, 1 = fp32
void launch_ipc_allreduce(const IpcAllReduceArgs& a, int dtype, hipStream_t s);

}  // namespace dtfe
