// torch.ops.dtfe.rccl_* : a native RCCL communicator owned by dtfe.
//
// torch.distributed's ProcessGroupNCCL runs every collective on its own internal
// stream and tracks it with a watchdog thread; it is not meant to be recorded into
// a hipGraph.  The data-parallel step of this framework is ONE hipGraph per step,
// so the gradient all-reduce must be a plain stream operation: these ops wrap
// ncclCommInitRank / ncclAllReduce (librccl, the copy torch itself links) and
// enqueue the collective on the caller's CURRENT stream.  The caller
// (parallel/rccl.py) forks a side stream off the compute stream for it, so in a
// captured graph the all-reduce is a node that runs concurrently with the rest of
// the backward pass and joins before the optimizer node.
//
// Communicators are created once per process (unique id exchanged over the c10d
// store by the Python side) and referenced by a small integer handle.
#include <ATen/ATen.h>
#include <ATen/hip/HIPContext.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <torch/library.h>

#include <algorithm>
#include <cstring>
#include <mutex>
#include <vector>

#include "../kernels/ipc_allreduce.h"

using at::Tensor;

namespace {

std::mutex g_mu;
std::vector<ncclComm_t> g_comms;

void rccl_check(ncclResult_t r, const char* what) {
  TORCH_CHECK(r == ncclSuccess, "dtfe: ", what, " failed: ", ncclGetErrorString(r));
}

ncclComm_t comm_of(int64_t h) {
  std::lock_guard<std::mutex> lk(g_mu);
  TORCH_CHECK(h >= 0 && h < (int64_t)g_comms.size() && g_comms[h] != nullptr, "dtfe: bad RCCL comm handle ", h);
  return g_comms[h];
}

ncclDataType_t rccl_dtype(const Tensor& t) {
  switch (t.scalar_type()) {
    case at::kFloat: return ncclFloat32;
    case at::kBFloat16: return ncclBfloat16;
    case at::kHalf: return ncclFloat16;
    case at::kInt: return ncclInt32;
    case at::kDouble: return ncclFloat64;
    default: TORCH_CHECK(false, "dtfe: unsupported RCCL dtype ", t.scalar_type());
  }
  return ncclFloat32;
}

ncclRedOp_t rccl_op(int64_t op) {
  switch (op) {
    case 0: return ncclSum;
    case 1: return ncclMax;
    case 2: return ncclMin;
    case 3: return ncclAvg;
    default: TORCH_CHECK(false, "dtfe: unsupported RCCL reduce op ", op);
  }
  return ncclSum;
}

int64_t rccl_id_bytes() { return (int64_t)sizeof(ncclUniqueId); }

Tensor rccl_unique_id() {
  ncclUniqueId id;
  rccl_check(ncclGetUniqueId(&id), "ncclGetUniqueId");
  Tensor t = at::empty({(int64_t)sizeof(id)}, at::TensorOptions().dtype(at::kByte));
  std::memcpy(t.data_ptr(), &id, sizeof(id));
  return t;
}

int64_t rccl_init(const Tensor& id, int64_t world, int64_t rank, int64_t device) {
  TORCH_CHECK(id.device().is_cpu() && id.scalar_type() == at::kByte && id.numel() == (int64_t)sizeof(ncclUniqueId),
              "dtfe: rccl_init expects the CPU uint8[", sizeof(ncclUniqueId), "] id of rccl_unique_id");
  TORCH_CHECK(world >= 1 && rank >= 0 && rank < world, "dtfe: bad rank ", rank, " / world ", world);
  ncclUniqueId uid;
  std::memcpy(&uid, id.contiguous().data_ptr(), sizeof(uid));
  TORCH_CHECK(hipSetDevice((int)device) == hipSuccess, "dtfe: hipSetDevice(", device, ") failed");
  ncclComm_t comm = nullptr;
  rccl_check(ncclCommInitRank(&comm, (int)world, uid, (int)rank), "ncclCommInitRank");
  std::lock_guard<std::mutex> lk(g_mu);
  g_comms.push_back(comm);
  return (int64_t)g_comms.size() - 1;
}

void rccl_all_reduce(Tensor buf, int64_t handle, int64_t op) {
  TORCH_CHECK(buf.is_cuda() && buf.is_contiguous(), "dtfe: rccl_all_reduce needs a contiguous GPU tensor");
  ncclComm_t comm = comm_of(handle);
  hipStream_t s = at::hip::getCurrentHIPStream().stream();
  rccl_check(ncclAllReduce(buf.data_ptr(), buf.data_ptr(), (size_t)buf.numel(), rccl_dtype(buf), rccl_op(op), comm, s),
             "ncclAllReduce");
}

void rccl_broadcast(Tensor buf, int64_t root, int64_t handle) {
  TORCH_CHECK(buf.is_cuda() && buf.is_contiguous(), "dtfe: rccl_broadcast needs a contiguous GPU tensor");
  ncclComm_t comm = comm_of(handle);
  hipStream_t s = at::hip::getCurrentHIPStream().stream();
  rccl_check(ncclBroadcast(buf.data_ptr(), buf.data_ptr(), (size_t)buf.numel(), rccl_dtype(buf), (int)root, comm, s),
             "ncclBroadcast");
}

// ncclCommGetAsyncError of the communicator: 0 = healthy, else the ncclResult_t code (a peer
// failed, a network / remote error surfaced).  Host-only, never blocks on the device: the comm
// watchdog (parallel/health.py CommWatchdog) polls it from its own thread.
int64_t rccl_status(int64_t handle) {
  ncclComm_t comm;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    if (handle < 0 || handle >= (int64_t)g_comms.size() || g_comms[handle] == nullptr) return -1;
    comm = g_comms[handle];
  }
  ncclResult_t async = ncclSuccess;
  const ncclResult_t r = ncclCommGetAsyncError(comm, &async);
  if (r != ncclSuccess) return (int64_t)r;
  return async == ncclInProgress ? 0 : (int64_t)async;
}

// ncclCommAbort: stops the communicator's in-flight collectives (a replayed graph blocked in an
// all-reduce whose peer died) and frees it.  The caller exits right after (a failed
// rank aborts the job; restart resumes from the checkpoint).
void rccl_abort(int64_t handle) {
  ncclComm_t comm;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    if (handle < 0 || handle >= (int64_t)g_comms.size()) return;
    comm = g_comms[handle];
    g_comms[handle] = nullptr;
  }
  if (comm != nullptr) (void)ncclCommAbort(comm);
}

void rccl_destroy(int64_t handle) {
  ncclComm_t comm;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    TORCH_CHECK(handle >= 0 && handle < (int64_t)g_comms.size(), "dtfe: bad RCCL comm handle ", handle);
    comm = g_comms[handle];
    g_comms[handle] = nullptr;
  }
  if (comm != nullptr) rccl_check(ncclCommDestroy(comm), "ncclCommDestroy");
}

// ------------------------------------------------------------------------------------
// hipIpc two-shot all-reduce (kernels/ipc_allreduce.hip).  Host side: one uncached
// exchange buffer per rank, its IPC handle exported, every peer's handle opened here.
struct IpcComm {
  int rank = 0, world = 1, device = 0;
  long cap = 0;
  char* local = nullptr;
  char* base[dtfe::IPC_MAXW] = {};
  bool opened[dtfe::IPC_MAXW] = {};
  uint32_t* epoch = nullptr;
  uint32_t* calls = nullptr;
  int* err = nullptr;
  double timeout_s = 30.0;
  int max_blocks = dtfe::IPC_MAXB;  // grid cap (ipc_set_max_blocks; identical on every rank)
  long cap_upto = -1;               // ... applied to launches of at most this many bytes (-1: all)
};
std::vector<IpcComm*> g_ipc;

void hip_check(hipError_t e, const char* what) {
  TORCH_CHECK(e == hipSuccess, "dtfe: ", what, " failed: ", hipGetErrorString(e));
}

IpcComm* ipc_of(int64_t h) {
  std::lock_guard<std::mutex> lk(g_mu);
  TORCH_CHECK(h >= 0 && h < (int64_t)g_ipc.size() && g_ipc[h] != nullptr, "dtfe: bad IPC comm handle ", h);
  return g_ipc[h];
}

int64_t ipc_create(int64_t cap_bytes, int64_t rank, int64_t world, int64_t device, double timeout_s) {
  TORCH_CHECK(world >= 1 && world <= dtfe::IPC_MAXW && rank >= 0 && rank < world, "dtfe: ipc world ", world,
              " rank ", rank, " (1..", dtfe::IPC_MAXW, " ranks)");
  auto* c = new IpcComm();
  c->rank = (int)rank;
  c->world = (int)world;
  c->device = (int)device;
  c->cap = (cap_bytes + 255) / 256 * 256;
  c->timeout_s = timeout_s;
  hip_check(hipSetDevice(c->device), "hipSetDevice");
  void* p = nullptr;
  const size_t bytes = (size_t)dtfe::IPC_DATA_OFF + 2 * (size_t)c->cap;
  hip_check(hipExtMallocWithFlags(&p, bytes, hipDeviceMallocUncached), "hipExtMallocWithFlags(uncached)");
  hip_check(hipMemset(p, 0, dtfe::IPC_DATA_OFF), "hipMemset(flags)");
  c->local = static_cast<char*>(p);
  c->base[c->rank] = c->local;
  hip_check(hipMalloc(reinterpret_cast<void**>(&c->epoch), dtfe::IPC_MAXB * sizeof(uint32_t) + 64), "hipMalloc");
  hip_check(hipMemset(c->epoch, 0, dtfe::IPC_MAXB * sizeof(uint32_t) + 64), "hipMemset");
  c->err = reinterpret_cast<int*>(c->epoch + dtfe::IPC_MAXB);
  c->calls = c->epoch + dtfe::IPC_MAXB + 4;
  hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
  std::lock_guard<std::mutex> lk(g_mu);
  g_ipc.push_back(c);
  return (int64_t)g_ipc.size() - 1;
}

Tensor ipc_handle(int64_t h) {
  IpcComm* c = ipc_of(h);
  hipIpcMemHandle_t mh;
  hip_check(hipIpcGetMemHandle(&mh, c->local), "hipIpcGetMemHandle");
  Tensor t = at::empty({(int64_t)sizeof(mh)}, at::TensorOptions().dtype(at::kByte));
  std::memcpy(t.data_ptr(), &mh, sizeof(mh));
  return t;
}

// handles: CPU uint8 [world, sizeof(hipIpcMemHandle_t)] (row r = rank r's handle)
void ipc_open(int64_t h, const Tensor& handles) {
  IpcComm* c = ipc_of(h);
  const int64_t hb = (int64_t)sizeof(hipIpcMemHandle_t);
  TORCH_CHECK(handles.device().is_cpu() && handles.scalar_type() == at::kByte && handles.dim() == 2 &&
                  handles.size(0) == c->world && handles.size(1) == hb,
              "dtfe: ipc_open expects uint8 [world, ", hb, "] handles");
  Tensor hc = handles.contiguous();
  hip_check(hipSetDevice(c->device), "hipSetDevice");
  for (int q = 0; q < c->world; ++q) {
    if (q == c->rank || c->opened[q]) continue;
    hipIpcMemHandle_t mh;
    std::memcpy(&mh, hc.data_ptr<uint8_t>() + q * hb, hb);
    void* p = nullptr;
    hip_check(hipIpcOpenMemHandle(&p, mh, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle");
    c->base[q] = static_cast<char*>(p);
    c->opened[q] = true;
  }
}

int64_t ipc_capacity(int64_t h) { return ipc_of(h)->cap; }

// workgroup cap of the launches of this comm of at most `upto_bytes` (-1: every launch; 1..IPC_MAXB):
// fewer workgroups hold fewer CUs while they wait for the peers (bench/ipc_interference.py); larger
// buffers keep the full grid.  Must be the same on every rank.
void ipc_set_max_blocks(int64_t h, int64_t n, int64_t upto_bytes) {
  TORCH_CHECK(n >= 1 && n <= dtfe::IPC_MAXB, "dtfe: ipc max_blocks must be 1..", dtfe::IPC_MAXB);
  ipc_of(h)->max_blocks = (int)n;
  ipc_of(h)->cap_upto = (long)upto_bytes;
}

void ipc_all_reduce(Tensor buf, int64_t h) {
  IpcComm* c = ipc_of(h);
  TORCH_CHECK(buf.is_cuda() && buf.is_contiguous() && buf.get_device() == c->device,
              "dtfe: ipc_all_reduce needs a contiguous tensor on the comm's GPU");
  TORCH_CHECK(buf.scalar_type() == at::kBFloat16 || buf.scalar_type() == at::kFloat,
              "dtfe: ipc_all_reduce supports bf16 / fp32");
  const long bytes = (long)buf.numel() * (long)buf.element_size();
  TORCH_CHECK(bytes + 64 <= c->cap, "dtfe: ipc_all_reduce of ", bytes, " B exceeds the staging capacity ", c->cap);
  for (int q = 0; q < c->world; ++q) TORCH_CHECK(c->base[q] != nullptr, "dtfe: ipc comm not opened (rank ", q, ")");
  if (buf.numel() == 0) return;
  dtfe::IpcAllReduceArgs a{};
  for (int q = 0; q < c->world; ++q) a.base[q] = c->base[q];
  a.cap = c->cap;
  a.rank = c->rank;
  a.world = c->world;
  a.buf = buf.data_ptr();
  a.n = buf.numel();
  a.epoch = c->epoch;
  a.calls = c->calls;
  a.err = c->err;
  a.timeout = (unsigned long long)(c->timeout_s * 1e8);  // wall_clock64: 100 MHz
  // the block count must be identical on every rank: a function of (n, world) only
  const long seg_vec = (bytes / 16 + c->world - 1) / c->world;
  long blocks = (seg_vec + 2 * dtfe::IPC_THREADS - 1) / (2 * dtfe::IPC_THREADS);
  const long cap = c->cap_upto < 0 || bytes <= c->cap_upto ? c->max_blocks : dtfe::IPC_MAXB;
  a.blocks = (int)std::max(1L, std::min(cap, blocks));
  dtfe::launch_ipc_allreduce(a, buf.scalar_type() == at::kBFloat16 ? 0 : 1,
                             at::hip::getCurrentHIPStream().stream());
}

// 0 = healthy, 1 = a barrier timed out (a peer never arrived).  Synchronizes the device.
int64_t ipc_status(int64_t h) {
  IpcComm* c = ipc_of(h);
  hip_check(hipSetDevice(c->device), "hipSetDevice");
  hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
  int e = 0;
  hip_check(hipMemcpy(&e, c->err, sizeof(int), hipMemcpyDeviceToHost), "hipMemcpy");
  return e;
}

void ipc_destroy(int64_t h) {
  IpcComm* c;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    TORCH_CHECK(h >= 0 && h < (int64_t)g_ipc.size(), "dtfe: bad IPC comm handle ", h);
    c = g_ipc[h];
    g_ipc[h] = nullptr;
  }
  if (c == nullptr) return;
  (void)hipSetDevice(c->device);
  (void)hipDeviceSynchronize();
  for (int q = 0; q < c->world; ++q)
    if (c->opened[q]) (void)hipIpcCloseMemHandle(c->base[q]);
  (void)hipFree(c->local);
  (void)hipFree(c->epoch);
  delete c;
}

}  // namespace

TORCH_LIBRARY_FRAGMENT(dtfe, m) {
  m.def("ipc_create(int cap_bytes, int rank, int world, int device, float timeout_s) -> int", &ipc_create);
  m.def("ipc_handle(int comm) -> Tensor", &ipc_handle);
  m.def("ipc_open(int comm, Tensor handles) -> ()", &ipc_open);
  m.def("ipc_capacity(int comm) -> int", &ipc_capacity);
  m.def("ipc_set_max_blocks(int comm, int n, int upto_bytes=-1) -> ()", &ipc_set_max_blocks);
  m.def("ipc_all_reduce(Tensor(a!) buf, int comm) -> ()", &ipc_all_reduce);
  m.def("ipc_status(int comm) -> int", &ipc_status);
  m.def("ipc_destroy(int comm) -> ()", &ipc_destroy);
  m.def("rccl_id_bytes() -> int", &rccl_id_bytes);
  m.def("rccl_unique_id() -> Tensor", &rccl_unique_id);
  m.def("rccl_init(Tensor id, int world, int rank, int device) -> int", &rccl_init);
  m.def("rccl_all_reduce(Tensor(a!) buf, int comm, int op) -> ()", &rccl_all_reduce);
  m.def("rccl_broadcast(Tensor(a!) buf, int root, int comm) -> ()", &rccl_broadcast);
  m.def("rccl_destroy(int comm) -> ()", &rccl_destroy);
  m.def("rccl_status(int comm) -> int", &rccl_status);
  m.def("rccl_abort(int comm) -> ()", &rccl_abort);
}
