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

#include <cstring>
#include <mutex>
#include <vector>

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

}  // namespace

TORCH_LIBRARY_FRAGMENT(dtfe, m) {
  m.def("rccl_id_bytes() -> int", &rccl_id_bytes);
  m.def("rccl_unique_id() -> Tensor", &rccl_unique_id);
  m.def("rccl_init(Tensor id, int world, int rank, int device) -> int", &rccl_init);
  m.def("rccl_all_reduce(Tensor(a!) buf, int comm, int op) -> ()", &rccl_all_reduce);
  m.def("rccl_broadcast(Tensor(a!) buf, int root, int comm) -> ()", &rccl_broadcast);
  m.def("rccl_destroy(int comm) -> ()", &rccl_destroy);
}
