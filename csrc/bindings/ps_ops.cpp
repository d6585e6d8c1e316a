// torch.ops.dtfe.ps_* : the native parameter-server data plane.
//
// Replaces TF's RecvTensor path (gan/distributed_gan.py:193 - every sess.run pulls the
// variables from and pushes the gradients to the ps task over gRPC) for a single node:
//
//   * shared page   - POSIX shm created by the ps task, mapped + hipHostRegister'ed by it and
//                     by every worker: one 128-B request/reply slot per worker (ps_link.h).
//   * IPC buffers   - the ps allocates, per worker, a gradient mailbox and a parameter reply
//                     buffer in its GPU's memory (uncached) and exports one hipIpc handle;
//                     workers map it and move bytes with their own copy kernels over xGMI.
//   * service       - a C++ progress thread in the ps process (no Python, no GIL): it polls
//                     the shared page, and for every request enqueues on its HIP stream the
//                     fused TF1 apply of the mailbox (every optimizer group of the shard), the
//                     reply snapshot (bf16 working copies + fp32 non-bf16 variables) and the
//                     reply store.  Async mode serialises applies in arrival order (one
//                     stream); --hogwild gives every worker its own stream (TF use_locking=False);
//                     sync mode accumulates replicas_to_aggregate fresh gradients (stale ones
//                     dropped) and applies their mean (SyncReplicasOptimizer semantics).
//   * control       - INIT / SAVE / SET_STATE / STATUS / DONE stay on the gloo channel
//                     (parallel/ps.py); those handlers pause the service around their access.
#include <ATen/ATen.h>
#include <ATen/hip/HIPContext.h>
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <torch/library.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstring>
#include <deque>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../kernels/optim.h"
#include "../kernels/ps_link.h"

using at::Tensor;

namespace {

void hchk(hipError_t e, const char* what) { TORCH_CHECK(e == hipSuccess, "dtfe ps: ", what, ": ", hipGetErrorString(e)); }

hipStream_t cur_stream() { return at::hip::getCurrentHIPStream().stream(); }

std::mutex g_mu;

// ------------------------------------------------------------------ shared page
struct Shm {
  std::string name;
  size_t bytes = 0;
  void* host = nullptr;
  void* dev = nullptr;
  bool owner = false;
};
std::vector<Shm*> g_shm;

Shm* shm_of(int64_t h) {
  std::lock_guard<std::mutex> lk(g_mu);
  TORCH_CHECK(h >= 0 && h < (int64_t)g_shm.size() && g_shm[h], "dtfe ps: bad shm handle ", h);
  return g_shm[h];
}

int64_t shm_map(const std::string& name, int64_t bytes, bool create) {
  auto* s = new Shm();
  s->name = name;
  s->bytes = (size_t)((bytes + 4095) / 4096 * 4096);
  s->owner = create;
  const int fd = create ? shm_open(name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600) : shm_open(name.c_str(), O_RDWR, 0600);
  TORCH_CHECK(fd >= 0, "dtfe ps: shm_open(", name, ") failed: ", strerror(errno));
  if (create) TORCH_CHECK(ftruncate(fd, (off_t)s->bytes) == 0, "dtfe ps: ftruncate failed");
  s->host = mmap(nullptr, s->bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  TORCH_CHECK(s->host != MAP_FAILED, "dtfe ps: mmap failed");
  if (create) std::memset(s->host, 0, s->bytes);
  hchk(hipHostRegister(s->host, s->bytes, hipHostRegisterMapped | hipHostRegisterPortable), "hipHostRegister");
  hchk(hipHostGetDevicePointer(&s->dev, s->host, 0), "hipHostGetDevicePointer");
  std::lock_guard<std::mutex> lk(g_mu);
  g_shm.push_back(s);
  return (int64_t)g_shm.size() - 1;
}

int64_t ps_shm_create(std::string name, int64_t bytes) { return shm_map(name, bytes, true); }
int64_t ps_shm_open(std::string name, int64_t bytes) { return shm_map(name, bytes, false); }

void ps_shm_close(int64_t h) {
  Shm* s;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    TORCH_CHECK(h >= 0 && h < (int64_t)g_shm.size(), "dtfe ps: bad shm handle");
    s = g_shm[h];
    g_shm[h] = nullptr;
  }
  if (!s) return;
  (void)hipHostUnregister(s->host);
  munmap(s->host, s->bytes);
  if (s->owner) shm_unlink(s->name.c_str());
  delete s;
}

uint64_t* slot_host(Shm* s, int w) { return reinterpret_cast<uint64_t*>(s->host) + (size_t)w * dtfe::PS_SLOT_WORDS; }
uint64_t* slot_dev(Shm* s, int w) { return reinterpret_cast<uint64_t*>(s->dev) + (size_t)w * dtfe::PS_SLOT_WORDS; }

// (req_seq, req_kind, req_tag, rep_seq, rep_gs, rep_ver, rep_stale) of worker w, read by the host
Tensor ps_shm_slot(int64_t h, int64_t w) {
  Shm* s = shm_of(h);
  TORCH_CHECK(w >= 0 && w < dtfe::PS_MAX_WORKERS, "dtfe ps: worker slot out of range");
  auto* p = slot_host(s, (int)w);
  Tensor t = at::empty({7}, at::TensorOptions().dtype(at::kLong));
  int64_t* o = t.data_ptr<int64_t>();
  auto rd = [&](int i) { return (int64_t)__atomic_load_n(p + i, __ATOMIC_ACQUIRE); };
  o[0] = rd(dtfe::PS_REQ_SEQ); o[1] = rd(dtfe::PS_REQ_KIND); o[2] = rd(dtfe::PS_REQ_TAG);
  o[3] = rd(dtfe::PS_REP_SEQ); o[4] = rd(dtfe::PS_REP_GS); o[5] = rd(dtfe::PS_REP_VER); o[6] = rd(dtfe::PS_REP_STALE);
  return t;
}

// host spin until worker w's reply number reaches `seq` (or timeout): returns (rep_gs, rep_ver), or raises
Tensor ps_shm_wait_reply(int64_t h, int64_t w, int64_t seq, double timeout_s) {
  Shm* s = shm_of(h);
  auto* p = slot_host(s, (int)w);
  const auto t0 = std::chrono::steady_clock::now();
  int spins = 0;
  while ((int64_t)__atomic_load_n(p + dtfe::PS_REP_SEQ, __ATOMIC_ACQUIRE) < seq) {
    if (++spins > 256) {
      spins = 0;
      sched_yield();
      const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      TORCH_CHECK(el < timeout_s, "dtfe ps: no reply from the parameter server within ", timeout_s, " s");
    }
  }
  Tensor t = at::empty({2}, at::TensorOptions().dtype(at::kLong));
  t.data_ptr<int64_t>()[0] = (int64_t)__atomic_load_n(p + dtfe::PS_REP_GS, __ATOMIC_ACQUIRE);
  t.data_ptr<int64_t>()[1] = (int64_t)__atomic_load_n(p + dtfe::PS_REP_VER, __ATOMIC_ACQUIRE);
  return t;
}

// ------------------------------------------------------------------ IPC buffers
struct IpcBuf {
  void* ptr = nullptr;
  bool owner = false;
  int device = 0;
};
std::vector<IpcBuf*> g_buf;

IpcBuf* buf_of(int64_t h) {
  std::lock_guard<std::mutex> lk(g_mu);
  TORCH_CHECK(h >= 0 && h < (int64_t)g_buf.size() && g_buf[h], "dtfe ps: bad buffer handle ", h);
  return g_buf[h];
}

int64_t ps_ipc_alloc(int64_t bytes, int64_t device) {
  auto* b = new IpcBuf();
  b->owner = true;
  b->device = (int)device;
  hchk(hipSetDevice(b->device), "hipSetDevice");
  hchk(hipExtMallocWithFlags(&b->ptr, (size_t)bytes, hipDeviceMallocUncached), "hipExtMallocWithFlags(uncached)");
  hchk(hipMemset(b->ptr, 0, (size_t)bytes), "hipMemset");
  hchk(hipDeviceSynchronize(), "hipDeviceSynchronize");
  std::lock_guard<std::mutex> lk(g_mu);
  g_buf.push_back(b);
  return (int64_t)g_buf.size() - 1;
}

Tensor ps_ipc_handle(int64_t h) {
  IpcBuf* b = buf_of(h);
  hipIpcMemHandle_t mh;
  hchk(hipIpcGetMemHandle(&mh, b->ptr), "hipIpcGetMemHandle");
  Tensor t = at::empty({(int64_t)sizeof(mh)}, at::TensorOptions().dtype(at::kByte));
  std::memcpy(t.data_ptr(), &mh, sizeof(mh));
  return t;
}

int64_t ps_ipc_open(const Tensor& handle, int64_t device) {
  TORCH_CHECK(handle.device().is_cpu() && handle.numel() == (int64_t)sizeof(hipIpcMemHandle_t),
              "dtfe ps: ipc handle must be CPU uint8[", sizeof(hipIpcMemHandle_t), "]");
  auto* b = new IpcBuf();
  b->device = (int)device;
  hipIpcMemHandle_t mh;
  std::memcpy(&mh, handle.contiguous().data_ptr(), sizeof(mh));
  hchk(hipSetDevice(b->device), "hipSetDevice");
  hchk(hipIpcOpenMemHandle(&b->ptr, mh, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle");
  std::lock_guard<std::mutex> lk(g_mu);
  g_buf.push_back(b);
  return (int64_t)g_buf.size() - 1;
}

int64_t ps_ipc_ptr(int64_t h) { return (int64_t)reinterpret_cast<uintptr_t>(buf_of(h)->ptr); }

void ps_ipc_close(int64_t h) {
  IpcBuf* b;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    TORCH_CHECK(h >= 0 && h < (int64_t)g_buf.size(), "dtfe ps: bad buffer handle");
    b = g_buf[h];
    g_buf[h] = nullptr;
  }
  if (!b) return;
  (void)hipSetDevice(b->device);
  (void)hipDeviceSynchronize();
  if (b->owner) (void)hipFree(b->ptr);
  else (void)hipIpcCloseMemHandle(b->ptr);
  delete b;
}

// ------------------------------------------------------------------ copy plans
// segs: CPU int64 [n, 4] = (src address, dst address, elements, mode); chunk elements per work item.
// Returns the device blob [PsSeg...][pad][PsWork...]; nwork via ps_plan_nwork.
int64_t plan_nwork(const Tensor& segs, int64_t chunk) {
  int64_t nw = 0;
  auto S = segs.contiguous();
  const int64_t* s = S.data_ptr<int64_t>();
  for (int64_t i = 0; i < S.size(0); ++i) nw += (s[i * 4 + 2] + chunk - 1) / chunk;
  return nw;
}

Tensor ps_plan(const Tensor& segs, int64_t chunk, const Tensor& device_like) {
  TORCH_CHECK(segs.device().is_cpu() && segs.scalar_type() == at::kLong && segs.dim() == 2 && segs.size(1) == 4,
              "dtfe ps: plan segs must be CPU int64 [n, 4]");
  TORCH_CHECK(chunk > 0 && chunk % 8 == 0, "dtfe ps: chunk must be a positive multiple of 8");
  auto S = segs.contiguous();
  const int64_t n = S.size(0);
  const int64_t* s = S.data_ptr<int64_t>();
  std::vector<dtfe::PsSeg> sg((size_t)n);
  std::vector<dtfe::PsWork> wk;
  for (int64_t i = 0; i < n; ++i) {
    sg[i].src = reinterpret_cast<const void*>((uintptr_t)s[i * 4 + 0]);
    sg[i].dst = reinterpret_cast<void*>((uintptr_t)s[i * 4 + 1]);
    sg[i].n = (long)s[i * 4 + 2];
    sg[i].mode = (int)s[i * 4 + 3];
    TORCH_CHECK(sg[i].mode >= 0 && sg[i].mode <= 5, "dtfe ps: bad copy mode");
    TORCH_CHECK(((s[i * 4 + 0] | s[i * 4 + 1]) & 15) == 0, "dtfe ps: copy segments must be 16-B aligned");
    for (long st = 0; st < sg[i].n; st += chunk) wk.push_back({(int)i, 0, st, std::min<long>(chunk, sg[i].n - st)});
  }
  const size_t bs = sg.size() * sizeof(dtfe::PsSeg), off = (bs + 255) / 256 * 256;
  Tensor host = at::zeros({(int64_t)(off + wk.size() * sizeof(dtfe::PsWork) + 16)}, at::TensorOptions().dtype(at::kByte));
  if (bs) std::memcpy(host.data_ptr<uint8_t>(), sg.data(), bs);
  if (!wk.empty()) std::memcpy(host.data_ptr<uint8_t>() + off, wk.data(), wk.size() * sizeof(dtfe::PsWork));
  return host.to(device_like.device());
}

const dtfe::PsSeg* plan_segs(const Tensor& blob) { return reinterpret_cast<const dtfe::PsSeg*>(blob.data_ptr()); }
const dtfe::PsWork* plan_work(const Tensor& blob, int64_t nseg) {
  const size_t off = (nseg * sizeof(dtfe::PsSeg) + 255) / 256 * 256;
  return reinterpret_cast<const dtfe::PsWork*>(reinterpret_cast<const uint8_t*>(blob.data_ptr()) + off);
}

void ps_copy(const Tensor& blob, int64_t nseg, int64_t nwork) {
  TORCH_CHECK(blob.is_cuda(), "dtfe ps: copy plan must be on the GPU");
  dtfe::launch_ps_copy(plan_segs(blob), plan_work(blob, nseg), (int)nwork, cur_stream());
}

// ------------------------------------------------------------------ worker side
void ps_request(int64_t shm, int64_t w, Tensor ctr, const c10::optional<Tensor>& ver, int64_t kind, int64_t shard,
                int64_t bump) {
  Shm* s = shm_of(shm);
  TORCH_CHECK(ctr.is_cuda() && ctr.scalar_type() == at::kLong, "dtfe ps: request counter must be a GPU int64");
  const bool hv = ver.has_value() && ver->defined();
  TORCH_CHECK(!hv || (ver->scalar_type() == at::kLong && shard >= 0 && shard < ver->numel()),
              "dtfe ps: ver must be a GPU int64 with one version per shard");
  const int64_t* v = hv ? ver->data_ptr<int64_t>() + shard : nullptr;
  dtfe::launch_ps_request(slot_dev(s, (int)w), ctr.data_ptr<int64_t>(), v, (int)kind, bump ? 1 : 0, cur_stream());
}

void ps_bucket(int64_t shm, int64_t w, const Tensor& ctr, int64_t b, int64_t lo, int64_t hi) {
  Shm* s = shm_of(shm);
  TORCH_CHECK(b >= 0 && b < dtfe::PS_MAX_BUCKETS, "dtfe ps: bucket index out of range");
  TORCH_CHECK(ctr.is_cuda() && ctr.scalar_type() == at::kLong, "dtfe ps: request counter must be a GPU int64");
  dtfe::launch_ps_bucket(slot_dev(s, (int)w), ctr.data_ptr<int64_t>(), (int)b, (long)lo, (long)hi, cur_stream());
}

void ps_wait(std::vector<int64_t> shms, int64_t w, int64_t gs_slot, const Tensor& ctr, const c10::optional<Tensor>& gs_out,
             const c10::optional<Tensor>& ver_out, Tensor err, double timeout_s) {
  TORCH_CHECK(!shms.empty() && shms.size() <= (size_t)dtfe::PS_MAX_SHARDS, "dtfe ps: 1..8 shards");
  dtfe::PsWaitArgs a{};
  for (size_t i = 0; i < shms.size(); ++i) a.slot[i] = slot_dev(shm_of(shms[i]), (int)w);
  a.nslots = (int)shms.size();
  a.gs_slot = (int)gs_slot;
  a.ctr = ctr.data_ptr<int64_t>();
  a.gs_out = (gs_out.has_value() && gs_out->defined()) ? gs_out->data_ptr<int32_t>() : nullptr;
  a.ver_out = (ver_out.has_value() && ver_out->defined()) ? ver_out->data_ptr<int64_t>() : nullptr;
  TORCH_CHECK(!a.ver_out || ver_out->numel() >= (int64_t)shms.size(), "dtfe ps: ver_out needs one entry per shard");
  a.err = err.data_ptr<int>();
  a.timeout_ticks = (unsigned long long)(timeout_s * 1e8);
  dtfe::launch_ps_wait(a, cur_stream());
}

// ------------------------------------------------------------------ ps service
// A partial plan of one optimizer group: its work items whose variable lies in a shard-flat range
// (a push bucket), same segment table.  Built on first use, cached by range.
struct SubPlan {
  Tensor blob;
  int nwork = 0;
};
struct Group {
  dtfe::OptArgs args;    // g / g16 and done_counter set per launch
  bool g16;
  std::vector<dtfe::OptSeg> hsegs;   // host copies of the plan (for the bucket sub-plans)
  std::vector<dtfe::OptWork> hwork;
  std::map<std::pair<long, long>, SubPlan> sub;
};
struct WorkerCh {
  void* mailbox = nullptr;       // this worker's gradient mailbox (ps GPU)
  Tensor snap;                   // reply snapshot plan (ps params -> reply buffer)
  int64_t snap_nseg = 0, snap_nwork = 0;
  // per-range snapshots (async bucketed pushes): host copy of the snapshot segments with each
  // one's shard-flat variable offset; a bucket's variables are copied into the reply buffer right
  // after its apply, so the reply itself only waits for the last bucket's copy
  std::vector<dtfe::PsSeg> snap_hsegs;
  std::vector<long> snap_off;
  std::map<std::pair<long, long>, SubPlan> snap_sub;
  uint64_t handled = 0;
  hipStream_t stream = nullptr;  // hogwild: per-worker stream
  std::vector<uint32_t*> done;   // per-group done counters (this channel's launches)
  bool waiting = false;          // sync mode: accumulated, reply pending
  uint64_t wait_seq = 0;
  // async bucket applies of the coming request: last bucket sequence applied per bucket, and the
  // ranges applied for request `range_seq`
  uint64_t bkt_done[dtfe::PS_MAX_BUCKETS] = {};
  uint64_t range_seq = 0;
  std::vector<std::pair<long, long>> ranges;
  std::vector<uint64_t> range_stamp;  // apply stamp of each entry of `ranges` (Service::stamp)
  // fused replies: per optimizer group, this worker's copy of the group's plan segments with the
  // second destinations (w16b / wt16b / pb) aimed at its reply buffer - the apply writes the
  // reply itself, no snapshot copy; sub-plans by shard range.  Empty: snapshot copies instead.
  bool fused = false;
  std::vector<std::vector<dtfe::OptSeg>> rsegs;
  std::vector<std::map<std::pair<long, long>, SubPlan>> rsub;
};
struct Service {
  Shm* shm = nullptr;
  int device = 0, nworkers = 0;
  bool sync = false, hogwild = false;
  int R = 1;
  std::vector<Group> groups;
  std::vector<WorkerCh> ch;
  const int32_t* gs = nullptr;
  long total = 0;                // shard-flat elements (bucket ranges are clamped to it)
  float* acc = nullptr;          // sync mode accumulator (fp32, shard layout)
  long acc_n = 0;
  int acc_count = 0;
  uint64_t version = 0;
  // async pulls stay current: every range apply gets a stamp and goes into `log` (bounded); a
  // worker's bucket range whose reply values were captured at its own apply is re-copied at its
  // request if another worker applied an overlapping range since (refresh_stale_ranges)
  struct ApplyRec {
    long lo, hi;
    uint64_t stamp;
    int w;
  };
  uint64_t stamp = 0;
  std::deque<ApplyRec> log;
  bool fused_replies = true;     // ps_service_set_fused (tests: the snapshot-copy path)
  // the apply stream on a GPU it shares with a worker (ps_service_set_stream): 1 = the device's
  // highest queue priority (its workgroups are dispatched ahead of the worker's as CUs free up);
  // cu_slice > 0 = a CU mask of that many CUs (hipExtStreamCreateWithCUMask)
  int stream_prio = 0, cu_slice = 0;
  hipStream_t stream = nullptr;
  std::thread th;
  std::atomic<bool> stop{false}, pause{false}, paused{false};
  std::atomic<int64_t> n_req{0}, n_apply{0}, n_stale{0}, n_bucket{0}, n_refresh{0};
  std::string error;
};
std::vector<Service*> g_svc;

Service* svc_of(int64_t h) {
  std::lock_guard<std::mutex> lk(g_mu);
  TORCH_CHECK(h >= 0 && h < (int64_t)g_svc.size() && g_svc[h], "dtfe ps: bad service handle ", h);
  return g_svc[h];
}

int64_t ps_service_create(int64_t shm, int64_t nworkers, int64_t device, bool sync, int64_t R, bool hogwild) {
  TORCH_CHECK(nworkers >= 1 && nworkers <= dtfe::PS_MAX_WORKERS, "dtfe ps: 1..", dtfe::PS_MAX_WORKERS, " workers");
  auto* s = new Service();
  s->shm = shm_of(shm);
  s->device = (int)device;
  s->nworkers = (int)nworkers;
  s->sync = sync;
  s->R = (int)std::max<int64_t>(1, R);
  s->hogwild = hogwild && !sync;
  s->ch.resize((size_t)nworkers);
  std::lock_guard<std::mutex> lk(g_mu);
  g_svc.push_back(s);
  return (int64_t)g_svc.size() - 1;
}

void ps_service_add_group(int64_t h, int64_t kind, Tensor p, const c10::optional<Tensor>& s1,
                          const c10::optional<Tensor>& s2, double lr, double beta1, double beta2, double eps,
                          double momentum, double rho, const c10::optional<Tensor>& beta_pow,
                          const c10::optional<Tensor>& global_step, int64_t gs_inc, const Tensor& blob, int64_t nseg,
                          int64_t nwork, bool g16) {
  Service* s = svc_of(h);
  Group g{};
  auto& a = g.args;
  a.kind = (int)kind;
  a.p = p.data_ptr<float>();
  a.gscale = 1.f;
  a.s1 = (s1.has_value() && s1->defined()) ? s1->data_ptr<float>() : nullptr;
  a.s2 = (s2.has_value() && s2->defined()) ? s2->data_ptr<float>() : nullptr;
  a.lr = (float)lr; a.beta1 = (float)beta1; a.beta2 = (float)beta2; a.eps = (float)eps;
  a.momentum = (float)momentum; a.rho = (float)rho;
  a.beta_pow = (beta_pow.has_value() && beta_pow->defined()) ? beta_pow->data_ptr<float>() : nullptr;
  a.global_step = (global_step.has_value() && global_step->defined()) ? global_step->data_ptr<int32_t>() : nullptr;
  a.gs_inc = (int)gs_inc;
  const size_t bs = (size_t)nseg * sizeof(dtfe::OptSeg), off = (bs + 255) / 256 * 256;
  a.segs = reinterpret_cast<const dtfe::OptSeg*>(blob.data_ptr());
  a.work = reinterpret_cast<const dtfe::OptWork*>((const char*)blob.data_ptr() + off);
  a.nwork = (int)nwork;
  g.g16 = g16;
  g.hsegs.resize((size_t)nseg);
  g.hwork.resize((size_t)nwork);
  if (nseg) hchk(hipMemcpy(g.hsegs.data(), a.segs, bs, hipMemcpyDeviceToHost), "plan segs D2H");
  if (nwork) hchk(hipMemcpy(g.hwork.data(), a.work, (size_t)nwork * sizeof(dtfe::OptWork), hipMemcpyDeviceToHost), "plan work D2H");
  s->groups.push_back(g);
}

void ps_service_set_worker(int64_t h, int64_t w, int64_t mailbox_addr, const Tensor& snap, int64_t snap_nseg,
                           int64_t snap_nwork) {
  Service* s = svc_of(h);
  TORCH_CHECK(w >= 0 && w < s->nworkers, "dtfe ps: worker index out of range");
  auto& c = s->ch[(size_t)w];
  c.mailbox = reinterpret_cast<void*>((uintptr_t)mailbox_addr);
  c.snap = snap;
  c.snap_nseg = snap_nseg;
  c.snap_nwork = snap_nwork;
}

// shard-flat offset of each snapshot segment's variable (enables the per-bucket snapshots)
void ps_service_set_snap_offsets(int64_t h, int64_t w, const Tensor& offs) {
  Service* s = svc_of(h);
  TORCH_CHECK(w >= 0 && w < s->nworkers, "dtfe ps: worker index out of range");
  auto& c = s->ch[(size_t)w];
  TORCH_CHECK(offs.device().is_cpu() && offs.scalar_type() == at::kLong && offs.numel() == c.snap_nseg,
              "dtfe ps: one CPU int64 offset per snapshot segment");
  c.snap_hsegs.resize((size_t)c.snap_nseg);
  if (c.snap_nseg)
    hchk(hipMemcpy(c.snap_hsegs.data(), plan_segs(c.snap), (size_t)c.snap_nseg * sizeof(dtfe::PsSeg),
                   hipMemcpyDeviceToHost), "snap segs D2H");
  auto o = offs.contiguous();
  c.snap_off.assign(o.data_ptr<int64_t>(), o.data_ptr<int64_t>() + o.numel());
  c.snap_sub.clear();
}

void ps_service_set_gs(int64_t h, const Tensor& gs) { svc_of(h)->gs = gs.data_ptr<int32_t>(); }

void ps_service_set_total(int64_t h, int64_t total) { svc_of(h)->total = (long)total; }

void ps_service_set_acc(int64_t h, Tensor acc) {
  Service* s = svc_of(h);
  s->acc = acc.data_ptr<float>();
  s->acc_n = acc.numel();
}

void launch_apply(Service* s, WorkerCh& c, hipStream_t st, const void* grad, bool grad_is_acc, float gscale) {
  for (size_t gi = 0; gi < s->groups.size(); ++gi) {
    dtfe::OptArgs a = s->groups[gi].args;
    if (grad_is_acc || !s->groups[gi].g16) {
      a.g = reinterpret_cast<const float*>(grad);
      a.g16 = nullptr;
    } else {
      a.g = nullptr;
      a.g16 = reinterpret_cast<const dtfe::bf16*>(grad);
    }
    a.gscale = gscale;
    a.done_counter = c.done[gi];
    dtfe::launch_apply_gradients(a, st);
  }
}

// the sub-plan of group g over shard range [lo, hi) (every variable lies wholly inside or outside),
// over segment table `segs` (the group's own, or a worker's reply-aimed copy), cached in `cache`
const SubPlan& sub_plan_of(Service* s, const Group& g, const std::vector<dtfe::OptSeg>& segs,
                           std::map<std::pair<long, long>, SubPlan>& cache, long lo, long hi) {
  auto key = std::make_pair(lo, hi);
  auto it = cache.find(key);
  if (it != cache.end()) return it->second;
  std::vector<dtfe::OptWork> wk;
  for (const auto& w : g.hwork) {
    const long off = segs[(size_t)w.seg].off;
    if (off >= lo && off < hi) wk.push_back(w);
  }
  SubPlan p;
  p.nwork = (int)wk.size();
  const size_t bs = segs.size() * sizeof(dtfe::OptSeg), off = (bs + 255) / 256 * 256;
  std::vector<uint8_t> host(off + wk.size() * sizeof(dtfe::OptWork) + 16, 0);
  if (bs) std::memcpy(host.data(), segs.data(), bs);
  if (!wk.empty()) std::memcpy(host.data() + off, wk.data(), wk.size() * sizeof(dtfe::OptWork));
  p.blob = at::empty({(int64_t)host.size()}, at::TensorOptions().dtype(at::kByte).device(at::kCUDA, s->device));
  hchk(hipMemcpy(p.blob.data_ptr(), host.data(), host.size(), hipMemcpyHostToDevice), "apply sub-plan H2D");
  return cache.emplace(key, std::move(p)).first->second;
}
const SubPlan& sub_plan(Service* s, Group& g, long lo, long hi) { return sub_plan_of(s, g, g.hsegs, g.sub, lo, hi); }

// worker c's apply args of group gi over [lo, hi): its mailbox as the gradient, the reply-aimed
// segment table when the channel is fused (nwork == 0: nothing of the group in the range)
dtfe::OptArgs range_args(Service* s, WorkerCh& c, size_t gi, long lo, long hi) {
  Group& g = s->groups[gi];
  const SubPlan& p = c.fused ? sub_plan_of(s, g, c.rsegs[gi], c.rsub[gi], lo, hi) : sub_plan(s, g, lo, hi);
  dtfe::OptArgs a = g.args;
  if (g.g16) {
    a.g = nullptr;
    a.g16 = reinterpret_cast<const dtfe::bf16*>(c.mailbox);
  } else {
    a.g = reinterpret_cast<const float*>(c.mailbox);
    a.g16 = nullptr;
  }
  const size_t bs = g.hsegs.size() * sizeof(dtfe::OptSeg), off = (bs + 255) / 256 * 256;
  a.segs = reinterpret_cast<const dtfe::OptSeg*>(p.blob.data_ptr());
  a.work = reinterpret_cast<const dtfe::OptWork*>((const char*)p.blob.data_ptr() + off);
  a.nwork = p.nwork;
  a.gscale = 1.f;
  a.skip_advance = 1;
  a.done_counter = c.done[gi];
  return a;
}

// fused replies for worker c: every reply-buffer segment of its snapshot plan must be the second
// destination of some apply segment (bf16 natural / transposed copy, or an fp32 variable);
// otherwise the channel keeps the snapshot copies
void build_fused(Service* s, WorkerCh& c) {
  c.fused = false;
  c.rsegs.clear();
  c.rsub.clear();
  if (c.snap_hsegs.empty() || c.snap_off.empty()) return;
  std::vector<char> used(c.snap_hsegs.size(), 0);
  std::vector<std::vector<dtfe::OptSeg>> rs;
  for (const Group& g : s->groups) {
    std::vector<dtfe::OptSeg> segs = g.hsegs;
    for (auto& sg : segs) {
      for (size_t i = 0; i < c.snap_hsegs.size(); ++i) {
        const dtfe::PsSeg& ps = c.snap_hsegs[i];
        if (ps.mode == 2 && sg.w16 && ps.src == sg.w16) {
          sg.w16b = reinterpret_cast<dtfe::bf16*>(ps.dst);
          used[i] = 1;
        } else if (ps.mode == 2 && sg.wt16 && ps.src == sg.wt16) {
          sg.wt16b = reinterpret_cast<dtfe::bf16*>(ps.dst);
          used[i] = 1;
        } else if (ps.mode == 0 && ps.src == g.args.p + sg.off) {
          sg.pb = reinterpret_cast<float*>(ps.dst);
          used[i] = 1;
        }
      }
    }
    rs.push_back(std::move(segs));
  }
  for (char u : used)
    if (!u) return;
  c.rsegs = std::move(rs);
  c.rsub.resize(s->groups.size());
  c.fused = true;
}

// apply the mailbox over shard range [lo, hi) with every group, leaving the step scalars alone
void launch_apply_range(Service* s, WorkerCh& c, hipStream_t st, long lo, long hi) {
  for (size_t gi = 0; gi < s->groups.size(); ++gi) {
    Group& g = s->groups[gi];
    const SubPlan& p = sub_plan(s, g, lo, hi);
    if (p.nwork == 0) continue;
    dtfe::OptArgs a = g.args;
    if (g.g16) {
      a.g = nullptr;
      a.g16 = reinterpret_cast<const dtfe::bf16*>(c.mailbox);
    } else {
      a.g = reinterpret_cast<const float*>(c.mailbox);
      a.g16 = nullptr;
    }
    const size_t bs = g.hsegs.size() * sizeof(dtfe::OptSeg), off = (bs + 255) / 256 * 256;
    a.segs = reinterpret_cast<const dtfe::OptSeg*>(p.blob.data_ptr());
    a.work = reinterpret_cast<const dtfe::OptWork*>((const char*)p.blob.data_ptr() + off);
    a.nwork = p.nwork;
    a.gscale = 1.f;
    a.skip_advance = 1;
    a.done_counter = c.done[gi];
    dtfe::launch_apply_gradients(a, st);
  }
}

constexpr long SNAP_CHUNK = 16384;  // elements per copy work item (= ps_native.COPY_CHUNK)

// copy the variables of shard range [lo, hi) into worker c's reply buffer (sub-plan cached by range)
void snap_range(Service* s, WorkerCh& c, hipStream_t st, long lo, long hi) {
  auto key = std::make_pair(lo, hi);
  auto it = c.snap_sub.find(key);
  if (it == c.snap_sub.end()) {
    std::vector<dtfe::PsWork> wk;
    for (size_t i = 0; i < c.snap_hsegs.size(); ++i) {
      if (c.snap_off[i] < lo || c.snap_off[i] >= hi) continue;
      for (long e = 0; e < c.snap_hsegs[i].n; e += SNAP_CHUNK)
        wk.push_back({(int)i, 0, e, std::min<long>(SNAP_CHUNK, c.snap_hsegs[i].n - e)});
    }
    SubPlan p;
    p.nwork = (int)wk.size();
    const size_t bs = c.snap_hsegs.size() * sizeof(dtfe::PsSeg), off = (bs + 255) / 256 * 256;
    std::vector<uint8_t> host(off + wk.size() * sizeof(dtfe::PsWork) + 16, 0);
    if (bs) std::memcpy(host.data(), c.snap_hsegs.data(), bs);
    if (!wk.empty()) std::memcpy(host.data() + off, wk.data(), wk.size() * sizeof(dtfe::PsWork));
    p.blob = at::empty({(int64_t)host.size()}, at::TensorOptions().dtype(at::kByte).device(at::kCUDA, s->device));
    hchk(hipMemcpy(p.blob.data_ptr(), host.data(), host.size(), hipMemcpyHostToDevice), "snap plan H2D");
    it = c.snap_sub.emplace(key, std::move(p)).first;
  }
  const SubPlan& p = it->second;
  if (p.nwork > 0)
    dtfe::launch_ps_copy(plan_segs(p.blob), plan_work(p.blob, (int64_t)c.snap_hsegs.size()), p.nwork, st);
}

// a bucket's apply (and, with per-range snapshots, its reply copy; a fused channel's apply writes
// the reply buffer itself)
void apply_bucket(Service* s, WorkerCh& c, hipStream_t st, long lo, long hi) {
  if (c.fused) {
    for (size_t gi = 0; gi < s->groups.size(); ++gi) {
      dtfe::OptArgs a = range_args(s, c, gi, lo, hi);
      if (a.nwork > 0) dtfe::launch_apply_gradients(a, st);
    }
    return;
  }
  launch_apply_range(s, c, st, lo, hi);
  if (!c.snap_off.empty()) snap_range(s, c, st, lo, hi);
}

// fused channel, at the request: apply the ranges not applied yet with each group's step scalars
// advanced by its last launch and the reply words published by the last launch of all (or by one
// small advance + reply kernel when some group has nothing left to apply)
void finish_fused(Service* s, WorkerCh& c, int w, hipStream_t st, uint64_t seq, uint64_t ver,
                  const std::vector<std::pair<long, long>>& todo) {
  struct L {
    size_t gi;
    dtfe::OptArgs a;
  };
  std::vector<L> ls;
  for (const auto& r : todo)
    for (size_t gi = 0; gi < s->groups.size(); ++gi) {
      dtfe::OptArgs a = range_args(s, c, gi, r.first, r.second);
      if (a.nwork > 0) ls.push_back({gi, a});
    }
  std::vector<int> last(s->groups.size(), -1);
  for (size_t i = 0; i < ls.size(); ++i) last[ls[i].gi] = (int)i;
  bool every = true;
  for (int l : last) every = every && l >= 0;
  auto set_reply = [&](dtfe::OptArgs& a) {
    a.rep_slot = slot_dev(s->shm, w);
    a.rep_gs = s->gs;
    a.rep_seq = seq;
    a.rep_ver = ver;
    a.rep_stale = 0;
  };
  for (size_t i = 0; i < ls.size(); ++i) {
    dtfe::OptArgs a = ls[i].a;
    a.skip_advance = last[ls[i].gi] == (int)i ? 0 : 1;
    if (every && i + 1 == ls.size()) set_reply(a);
    dtfe::launch_apply_gradients(a, st);
  }
  if (every) return;
  std::vector<dtfe::OptArgs> adv;
  for (size_t gi = 0; gi < s->groups.size(); ++gi)
    if (last[gi] < 0) adv.push_back(s->groups[gi].args);
  set_reply(adv.back());
  dtfe::launch_opt_advance_reply(adv.data(), (int)adv.size(), st);
}

// a range apply of worker w (any path): its stamp, logged for refresh_stale_ranges
uint64_t note_apply(Service* s, int w, long lo, long hi) {
  const uint64_t t = ++s->stamp;
  if (s->nworkers > 1) {
    s->log.push_back({lo, hi, t, w});
    if (s->log.size() > 4096) s->log.pop_front();
  }
  return t;
}

// Worker w's bucket ranges were written into its reply buffer when ITS apply ran (fused: by the
// apply itself; snapshot path: the per-range copy right after it).  A range another worker applied
// since then would reach w's pull one update late - the reference's pull reads the variable's
// value at pull time (gan/distributed_gan.py:193) - so it is copied again now.  Every non-hogwild
// apply and copy runs on the service stream in issue order, so the copy reads the current values.
// (hogwild: the applies race by design; nothing to refresh against.)
void refresh_stale_ranges(Service* s, WorkerCh& c, int w, hipStream_t st) {
  if (s->nworkers < 2 || s->hogwild || c.snap_off.empty()) return;
  const uint64_t oldest = s->log.empty() ? 0 : s->log.front().stamp;
  for (size_t i = 0; i < c.ranges.size(); ++i) {
    const long lo = c.ranges[i].first, hi = c.ranges[i].second;
    const uint64_t t = i < c.range_stamp.size() ? c.range_stamp[i] : 0;
    bool stale = t < oldest;  // fell out of the log: copy conservatively
    for (auto it = s->log.rbegin(); !stale && it != s->log.rend() && it->stamp > t; ++it)
      stale = it->w != w && it->lo < hi && lo < it->hi;
    if (stale) {
      snap_range(s, c, st, lo, hi);
      s->n_refresh++;
    }
  }
}

// async push with buckets: apply every bucket range of request `seq` not applied yet (the gaps
// between the ranges already applied - all of the shard when the worker sent no bucket), then
// advance each group's step scalars once.  Returns true when the reply buffer is already current.
bool finish_bucketed(Service* s, WorkerCh& c, int w, hipStream_t st, uint64_t seq) {
  std::vector<std::pair<long, long>> done = c.range_seq == seq ? c.ranges : std::vector<std::pair<long, long>>{};
  if (!done.empty()) refresh_stale_ranges(s, c, w, st);
  std::sort(done.begin(), done.end());
  if (c.fused) {
    std::vector<std::pair<long, long>> todo;
    long at = 0;
    for (const auto& r : done) {
      if (r.first > at) todo.emplace_back(at, r.first);
      at = std::max(at, r.second);
    }
    if (at < s->total) todo.emplace_back(at, s->total);
    for (const auto& r : todo) note_apply(s, w, r.first, r.second);
    finish_fused(s, c, w, st, seq, s->version + 1, todo);
    c.ranges.clear();
    c.range_stamp.clear();
    return true;
  }
  long at = 0;
  for (const auto& r : done) {
    if (r.first > at) {
      apply_bucket(s, c, st, at, r.first);
      note_apply(s, w, at, r.first);
    }
    at = std::max(at, r.second);
  }
  if (at < s->total) {
    apply_bucket(s, c, st, at, s->total);
    note_apply(s, w, at, s->total);
  }
  for (const auto& g : s->groups) dtfe::launch_opt_advance(g.args, st);
  c.ranges.clear();
  c.range_stamp.clear();
  return !c.snap_off.empty();
}

void reply(Service* s, int w, hipStream_t st, uint64_t seq, int stale, bool snapped = false) {
  auto& c = s->ch[(size_t)w];
  if (!snapped && c.snap_nwork > 0)
    dtfe::launch_ps_copy(plan_segs(c.snap), plan_work(c.snap, c.snap_nseg), (int)c.snap_nwork, st);
  dtfe::launch_ps_reply(slot_dev(s->shm, w), s->gs, seq, s->version, stale, st);
}

// sync accumulator += mailbox (or = on the first contribution) via a one-segment copy plan
struct AccPlan {
  Tensor blob;
  int64_t nwork = 0;
};

hipStream_t make_service_stream(int prio, int cu_slice) {
  hipStream_t st = nullptr;
  if (cu_slice > 0) {
    int dev = 0, ncu = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    const int words = (ncu + 31) / 32;
    std::vector<uint32_t> mask((size_t)words, 0u);
    for (int i = 0; i < std::min(cu_slice, ncu); ++i) mask[(size_t)(i / 32)] |= 1u << (i % 32);
    if (hipExtStreamCreateWithCUMask(&st, (uint32_t)words, mask.data()) == hipSuccess) return st;
    st = nullptr;
  }
  if (prio > 0) {
    int lo = 0, hi = 0;
    (void)hipDeviceGetStreamPriorityRange(&lo, &hi);
    if (hipStreamCreateWithPriority(&st, hipStreamNonBlocking, hi) == hipSuccess) return st;
  }
  (void)hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
  return st;
}

void run(Service* s) {
  if (hipSetDevice(s->device) != hipSuccess) {
    s->error = "hipSetDevice failed";
    return;
  }
  // per-worker done counters (a launch's last-workgroup ticket must not be shared by concurrent launches)
  for (auto& c : s->ch) {
    for (size_t g = 0; g < s->groups.size(); ++g) {
      uint32_t* d = nullptr;
      if (hipMalloc(&d, 64) != hipSuccess || hipMemset(d, 0, 64) != hipSuccess) {
        s->error = "hipMalloc(done) failed";
        return;
      }
      c.done.push_back(d);
    }
    if (s->hogwild) (void)hipStreamCreateWithFlags(&c.stream, hipStreamNonBlocking);
  }
  s->stream = make_service_stream(s->stream_prio, s->cu_slice);
  (void)hipDeviceSynchronize();
  // accumulate plans for sync mode: mailbox(w) -> acc, mode first/add
  std::vector<AccPlan> acc_first, acc_add;
  auto mk = [&](void* src, int mode) {
    AccPlan p;
    dtfe::PsSeg sg{src, s->acc, s->acc_n, mode, 0};
    std::vector<dtfe::PsWork> wk;
    for (long st = 0; st < s->acc_n; st += 65536) wk.push_back({0, 0, st, std::min<long>(65536, s->acc_n - st)});
    const size_t off = 256;
    std::vector<uint8_t> host(off + wk.size() * sizeof(dtfe::PsWork) + 16, 0);
    std::memcpy(host.data(), &sg, sizeof(sg));
    std::memcpy(host.data() + off, wk.data(), wk.size() * sizeof(dtfe::PsWork));
    p.blob = at::empty({(int64_t)host.size()}, at::TensorOptions().dtype(at::kByte).device(at::kCUDA, s->device));
    hchk(hipMemcpy(p.blob.data_ptr(), host.data(), host.size(), hipMemcpyHostToDevice), "plan H2D");
    p.nwork = (int64_t)wk.size();
    return p;
  };
  if (s->sync && s->acc) {
    const bool g16 = !s->groups.empty() && s->groups[0].g16;
    for (auto& c : s->ch) {
      acc_first.push_back(mk(c.mailbox, g16 ? 3 : 0));
      acc_add.push_back(mk(c.mailbox, g16 ? 5 : 4));
    }
  }
  int idle = 0;
  while (!s->stop.load(std::memory_order_acquire)) {
    if (s->pause.load(std::memory_order_acquire)) {
      (void)hipStreamSynchronize(s->stream);
      for (auto& c : s->ch)
        if (c.stream) (void)hipStreamSynchronize(c.stream);
      s->paused.store(true, std::memory_order_release);
      while (s->pause.load(std::memory_order_acquire) && !s->stop.load(std::memory_order_acquire)) sched_yield();
      s->paused.store(false, std::memory_order_release);
      continue;
    }
    bool any = false;
    for (int w = 0; w < s->nworkers; ++w) {
      auto& c = s->ch[(size_t)w];
      uint64_t* sl = slot_host(s->shm, w);
      hipStream_t bst = c.stream ? c.stream : s->stream;
      // async: apply each pushed bucket as soon as it is announced (the worker is still in backward)
      auto scan_buckets = [&](uint64_t floor) {  // buckets of requests after `floor`
        for (int b = 0; b < dtfe::PS_MAX_BUCKETS; ++b) {
          const uint64_t bseq = __atomic_load_n(sl + dtfe::PS_BKT_BASE + 3 * b, __ATOMIC_ACQUIRE);
          if (bseq <= floor || bseq <= c.bkt_done[b]) continue;
          const long lo = std::max(0L, (long)__atomic_load_n(sl + dtfe::PS_BKT_BASE + 3 * b + 1, __ATOMIC_ACQUIRE));
          const long hi = std::min(s->total, (long)__atomic_load_n(sl + dtfe::PS_BKT_BASE + 3 * b + 2, __ATOMIC_ACQUIRE));
          c.bkt_done[b] = bseq;
          if (c.range_seq != bseq) {
            c.range_seq = bseq;
            c.ranges.clear();
            c.range_stamp.clear();
          }
          if (lo < hi) {
            apply_bucket(s, c, bst, lo, hi);
            c.ranges.emplace_back(lo, hi);
            c.range_stamp.push_back(note_apply(s, w, lo, hi));
            s->n_bucket++;
          }
          any = true;
        }
      };
      if (!s->sync && s->total > 0) scan_buckets(c.handled);
      const uint64_t seq = __atomic_load_n(sl + dtfe::PS_REQ_SEQ, __ATOMIC_ACQUIRE);
      if (seq == c.handled) continue;
      c.handled = seq;
      any = true;
      s->n_req++;
      const uint64_t kind = __atomic_load_n(sl + dtfe::PS_REQ_KIND, __ATOMIC_ACQUIRE);
      hipStream_t st = c.stream ? c.stream : s->stream;
      if (kind != dtfe::PS_PUSH) {  // pull only
        reply(s, w, st, seq, 0);
        continue;
      }
      if (!s->sync) {
        bool snapped = false;
        if (s->total > 0) {
          scan_buckets(seq - 1);  // bucket words published just before this request
          if (c.fused) {       // the apply publishes the reply itself
            finish_bucketed(s, c, w, st, seq);
            s->version++;
            s->n_apply++;
            continue;
          }
          snapped = finish_bucketed(s, c, w, st, seq);
        } else {
          launch_apply(s, c, st, c.mailbox, false, 1.f);
        }
        s->version++;
        s->n_apply++;
        reply(s, w, st, seq, 0, snapped);
        continue;
      }
      // sync: drop stale, accumulate fresh, apply the mean after R contributions
      const uint64_t tag = __atomic_load_n(sl + dtfe::PS_REQ_TAG, __ATOMIC_ACQUIRE);
      if (tag < s->version || !s->acc) {
        s->n_stale++;
        reply(s, w, st, seq, 1);
        continue;
      }
      const AccPlan& ap = s->acc_count == 0 ? acc_first[(size_t)w] : acc_add[(size_t)w];
      dtfe::launch_ps_copy(plan_segs(ap.blob), plan_work(ap.blob, 1), (int)ap.nwork, st);
      s->acc_count++;
      c.waiting = true;
      c.wait_seq = seq;
    }
    // sync: a round is complete once R fresh gradients are in - checked every pass, not only
    // on an arrival, so a target lowered by a departing worker releases the waiting ones
    if (s->sync && s->acc_count > 0 && s->acc_count >= s->R) {
      launch_apply(s, s->ch[0], s->stream, s->acc, true, 1.f / (float)s->acc_count);
      s->version++;
      s->n_apply++;
      s->acc_count = 0;
      any = true;
      for (int q = 0; q < s->nworkers; ++q) {
        auto& cq = s->ch[(size_t)q];
        if (!cq.waiting) continue;
        cq.waiting = false;
        reply(s, q, s->stream, cq.wait_seq, 0);
      }
    }
    if (!any) {
      if (++idle > 64) {
        idle = 0;
        sched_yield();
      }
    } else {
      idle = 0;
    }
  }
  (void)hipStreamSynchronize(s->stream);
  for (auto& c : s->ch) {
    if (c.stream) {
      (void)hipStreamSynchronize(c.stream);
      (void)hipStreamDestroy(c.stream);
    }
    for (auto* d : c.done) (void)hipFree(d);
    c.done.clear();
  }
  (void)hipStreamDestroy(s->stream);
}

// the apply stream's priority / CU slice (see Service::stream_prio); before start
void ps_service_set_stream(int64_t h, int64_t prio, int64_t cu_slice) {
  Service* s = svc_of(h);
  s->stream_prio = (int)prio;
  s->cu_slice = (int)cu_slice;
}

// fused replies (default) or the snapshot-copy path for every async channel; before start
void ps_service_set_fused(int64_t h, bool on) { svc_of(h)->fused_replies = on; }

void ps_service_start(int64_t h) {
  Service* s = svc_of(h);
  TORCH_CHECK(!s->groups.empty(), "dtfe ps: service has no optimizer group");
  for (auto& c : s->ch) TORCH_CHECK(c.mailbox != nullptr, "dtfe ps: every worker channel needs a mailbox");
  TORCH_CHECK(!s->sync || s->acc, "dtfe ps: sync mode needs an accumulator");
  // async channels with per-variable reply segments: replies written by the applies themselves
  if (!s->sync && s->fused_replies && (int)s->groups.size() <= dtfe::OPT_GROUP_MAX)
    for (auto& c : s->ch) build_fused(s, c);
  s->th = std::thread(run, s);
}

// pause: the service thread drains its streams and stops issuing work until resume (the
// control handlers - INIT, SAVE, SET_STATE - then read or rewrite the shard safely)
void ps_service_pause(int64_t h) {
  Service* s = svc_of(h);
  s->pause.store(true, std::memory_order_release);
  while (!s->paused.load(std::memory_order_acquire) && !s->stop.load() && s->th.joinable()) sched_yield();
}
void ps_service_resume(int64_t h) { svc_of(h)->pause.store(false, std::memory_order_release); }

Tensor ps_service_stats(int64_t h) {
  Service* s = svc_of(h);
  Tensor t = at::empty({6}, at::TensorOptions().dtype(at::kLong));
  t.data_ptr<int64_t>()[4] = s->n_bucket.load();
  t.data_ptr<int64_t>()[5] = s->n_refresh.load();
  t.data_ptr<int64_t>()[0] = s->n_req.load();
  t.data_ptr<int64_t>()[1] = s->n_apply.load();
  t.data_ptr<int64_t>()[2] = s->n_stale.load();
  t.data_ptr<int64_t>()[3] = (int64_t)s->version;
  return t;
}

// sync mode: a worker left for good (DONE / lost) - lower the aggregation target so the
// remaining ones are not held forever (must be called while paused or before start)
void ps_service_set_replicas(int64_t h, int64_t R) { svc_of(h)->R = (int)std::max<int64_t>(1, R); }

void ps_service_stop(int64_t h) {
  Service* s;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    TORCH_CHECK(h >= 0 && h < (int64_t)g_svc.size(), "dtfe ps: bad service handle");
    s = g_svc[h];
    g_svc[h] = nullptr;
  }
  if (!s) return;
  s->pause.store(false);
  s->stop.store(true, std::memory_order_release);
  if (s->th.joinable()) s->th.join();
  TORCH_CHECK(s->error.empty(), "dtfe ps service: ", s->error);
  delete s;
}

}  // namespace

TORCH_LIBRARY_FRAGMENT(dtfe, m) {
  m.def("ps_shm_create(str name, int bytes) -> int", &ps_shm_create);
  m.def("ps_shm_open(str name, int bytes) -> int", &ps_shm_open);
  m.def("ps_shm_close(int h) -> ()", &ps_shm_close);
  m.def("ps_shm_slot(int h, int w) -> Tensor", &ps_shm_slot);
  m.def("ps_shm_wait_reply(int h, int w, int seq, float timeout_s) -> Tensor", &ps_shm_wait_reply);
  m.def("ps_ipc_alloc(int bytes, int device) -> int", &ps_ipc_alloc);
  m.def("ps_ipc_handle(int h) -> Tensor", &ps_ipc_handle);
  m.def("ps_ipc_open(Tensor handle, int device) -> int", &ps_ipc_open);
  m.def("ps_ipc_ptr(int h) -> int", &ps_ipc_ptr);
  m.def("ps_ipc_close(int h) -> ()", &ps_ipc_close);
  m.def("ps_plan(Tensor segs, int chunk, Tensor device_like) -> Tensor", &ps_plan);
  m.def("ps_plan_nwork(Tensor segs, int chunk) -> int", &plan_nwork);
  m.def("ps_copy(Tensor blob, int nseg, int nwork) -> ()", &ps_copy);
  m.def("ps_request(int shm, int w, Tensor(a!) ctr, Tensor? ver, int kind, int shard=0, int bump=1) -> ()", &ps_request);
  m.def("ps_wait(int[] shms, int w, int gs_slot, Tensor ctr, Tensor(a!)? gs_out, Tensor(b!)? ver_out, Tensor(c!) err,"
        " float timeout_s) -> ()", &ps_wait);
  m.def("ps_service_create(int shm, int nworkers, int device, bool sync, int R, bool hogwild) -> int", &ps_service_create);
  m.def("ps_service_add_group(int h, int kind, Tensor(a!) p, Tensor(b!)? s1, Tensor(c!)? s2, float lr, float beta1,"
        " float beta2, float eps, float momentum, float rho, Tensor(d!)? beta_pow, Tensor(e!)? global_step, int gs_inc,"
        " Tensor blob, int nseg, int nwork, bool g16) -> ()", &ps_service_add_group);
  m.def("ps_service_set_worker(int h, int w, int mailbox_addr, Tensor snap, int snap_nseg, int snap_nwork) -> ()",
        &ps_service_set_worker);
  m.def("ps_service_set_total(int h, int total) -> ()", &ps_service_set_total);
  m.def("ps_service_set_snap_offsets(int h, int w, Tensor offs) -> ()", &ps_service_set_snap_offsets);
  m.def("ps_bucket(int shm, int w, Tensor ctr, int b, int lo, int hi) -> ()", &ps_bucket);
  m.def("ps_service_set_gs(int h, Tensor gs) -> ()", &ps_service_set_gs);
  m.def("ps_service_set_acc(int h, Tensor(a!) acc) -> ()", &ps_service_set_acc);
  m.def("ps_service_set_fused(int h, bool on) -> ()", &ps_service_set_fused);
  m.def("ps_service_set_stream(int h, int prio, int cu_slice) -> ()", &ps_service_set_stream);
  m.def("ps_service_start(int h) -> ()", &ps_service_start);
  m.def("ps_service_pause(int h) -> ()", &ps_service_pause);
  m.def("ps_service_resume(int h) -> ()", &ps_service_resume);
  m.def("ps_service_stats(int h) -> Tensor", &ps_service_stats);
  m.def("ps_service_set_replicas(int h, int R) -> ()", &ps_service_set_replicas);
  m.def("ps_service_stop(int h) -> ()", &ps_service_stop);
}
