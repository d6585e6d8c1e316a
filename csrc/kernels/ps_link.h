// Parameter-server data plane over hipIpc-mapped device memory.
//
// Every (ps shard, worker) pair owns a gradient mailbox and a parameter reply buffer in the
// ps GPU's memory (uncached, exported with hipIpcGetMemHandle, mapped by the worker); a push
// is the worker's GPU writing its gradients straight into the mailbox over xGMI (or locally
// when the worker shares the ps's GPU), a pull is its GPU reading the reply buffer.  The
// request / reply handshake lives in a small shared-memory page mapped into both processes and
// registered for device access: the worker's GPU publishes "request s" with a system-scope
// store once its push has completed, the ps's native service thread polls the page, enqueues the
// fused apply - which writes the worker's reply buffer and the reply words itself - on its own
// stream; the worker's GPU waits
// for the reply in a bounded spin kernel, then pulls.  No host round trip on the worker side,
// so the whole worker step (compute, push, request, wait, pull) replays as one hipGraph.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "common.h"

namespace dtfe {

// One copy segment (element counts; pointers may be local or peer-mapped device memory).
// mode: 0 f32->f32, 1 f32->bf16, 2 bf16->bf16, 3 bf16->f32, 4 f32 += f32, 5 f32 += bf16
struct PsSeg {
  const void* src;
  void* dst;
  long n;
  int mode;
  int pad;
};
struct PsWork {
  int seg;
  int pad;
  long start, count;
};

constexpr int PS_MAX_WORKERS = 64;
constexpr int PS_SLOT_WORDS = 32;  // 256 B per worker slot (own cache lines)
constexpr int PS_MAX_BUCKETS = 4;

// shared page layout (uint64 words): [worker w][PS_SLOT_WORDS] of
enum PsWord : int {
  PS_REQ_SEQ = 0,   // written last by the worker's GPU (request number, 1, 2, ...)
  PS_REQ_KIND = 1,  // 1 = push (apply the mailbox), 2 = pull only
  PS_REQ_TAG = 2,   // sync mode: shard version the gradient was computed from
  PS_REP_SEQ = 8,   // written last by the ps's GPU: the request number answered
  PS_REP_GS = 9,    // global step after the apply (the gs shard; -1 elsewhere)
  PS_REP_VER = 10,  // shard version after the apply
  PS_REP_STALE = 11, // 1 when a sync-mode gradient was dropped as stale
  // bucket b (< PS_MAX_BUCKETS) of the coming push: its gradient range [LO, HI) (shard-flat
  // elements) is in the mailbox; BKT_SEQ is written last = the request number it belongs to.
  // The ps applies the range as soon as it sees it (async mode), overlapping the worker's backward.
  PS_BKT_BASE = 16   // + 3b: BKT_SEQ, + 3b + 1: BKT_LO, + 3b + 2: BKT_HI
};
enum PsKind : int { PS_PUSH = 1, PS_PULL = 2 };

// worker GPU, after bucket b's push: slot[BKT_LO/HI(b)] = lo / hi; slot[BKT_SEQ(b)] = *ctr + 1 (release)
void launch_ps_bucket(uint64_t* slot, const int64_t* ctr, int b, long lo, long hi, hipStream_t s);

// the copy plan: nwork items over the segments (one launch)
void launch_ps_copy(const PsSeg* segs, const PsWork* work, int nwork, hipStream_t s);

// worker GPU: ctr += bump; slot[KIND] = kind; slot[TAG] = *ver; slot[REQ_SEQ] = ctr (release).
// An exchange with several shards bumps once (first shard) so every shard sees the same number.
void launch_ps_request(uint64_t* slot, int64_t* ctr, const int64_t* ver, int kind, int bump, hipStream_t s);

// worker GPU: spin (bounded by timeout_ticks of the 100 MHz wall clock) until every slot's
// REP_SEQ >= *ctr; then gs_out = slot[gs_slot][REP_GS], ver_out[k] = slot[k][REP_VER].  On a
// timeout *err = 1 and the kernel returns.
constexpr int PS_MAX_SHARDS = 8;
struct PsWaitArgs {
  uint64_t* slot[PS_MAX_SHARDS];  // this worker's slot in every ps shard's shared page
  int nslots, gs_slot;
  const int64_t* ctr;
  int32_t* gs_out;
  int64_t* ver_out;
  int* err;
  unsigned long long timeout_ticks;
};
void launch_ps_wait(const PsWaitArgs& a, hipStream_t s);

// ps GPU: slot[REP_GS] = gs ? *gs : -1; slot[REP_VER] = ver; slot[REP_STALE] = stale; slot[REP_SEQ] = seq
void launch_ps_reply(uint64_t* slot, const int32_t* gs, uint64_t seq, uint64_t ver, int stale, hipStream_t s);

}  // namespace dtfe
