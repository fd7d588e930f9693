// libmysti_verify.so: contexts, device sharding and the C ABI of include/mysti_verify.h.
//
// One mv_ctx owns, per HIP device: a stream; the fixed-base tables ([0..128]B and
// [0..128](2^124 B) for the ladders, the comb table C_B); the committee (keys, stakes, the
// per-key comb tables C_A); growable device / pinned-host buffers. Host-buffer calls split
// their items into one contiguous shard per device and run each shard on its own host
// thread (one stream per device, no collective: only per-item verdicts come back), in
// chunks of at most cfg.max_batch items. Calls on one ctx are serialised by a mutex.
#include <hip/hip_runtime.h>
#include <limits.h>
#include <linux/futex.h>
#include <sched.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <dirent.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <atomic>
#include <condition_variable>
#include <deque>
#include <memory>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/mysti_verify.h"
#include "block_codec.h"
#include "kernels.h"

namespace {

constexpr int kBlockStage0 = mvk::BATCH_STAGES;  // parse, hash, verify, verdict
constexpr int kGuardBatches = 64;  // batches cut into sub-batch equations after a failure
// Dense failures (config 3: ~1% of the signatures bad, so every sub-batch equation fails and the
// whole batch is re-verified after a wasted MSM): a guarded batch that failed in at least half
// of its groups sends the next kSingleRun batches straight to the single path. Each of those
// counts its rejected signatures; while a batch holds at least kDenseRejects of them the run is
// renewed, otherwise the equation is tried again (guarded). The run is longer than the batches a
// caller can have in flight (kFlagRing): a renewal is seen only when a single-path batch
// completes, and a run that ran out before then sent a batch back to a doomed equation (config
// 3 with three streams: 2 of 10 batches). Recovery does not wait for the run: the first clean
// single-path batch to complete ends it.
constexpr int kSingleRun = 32;
constexpr uint32_t kDenseRejects = 4;
constexpr uint32_t kSingleMark = 0x80000000u;  // flag_groups entry of a single-path batch
constexpr int kBlockStages = 4;
constexpr int kWalStage0 = kBlockStage0 + kBlockStages;  // walk, crc
static_assert(kWalStage0 + 2 == MV_NSTAGES, "stage count");

// Buffers that grow retire the old allocation instead of freeing it at once: hipFree /
// hipHostFree drain the whole device, which would wait for the resident online kernel (it lives
// while online traffic flows) and for every other stream's calls. A retired block may still be
// read by work in flight: `guard` (when set) is the completion event of the ring slot it served,
// recorded after every call that used the slot, so its completion means no call still reads it
// (a later record on the same slot completes later still); blocks without a guard served only
// synchronous host-buffer calls, which had finished when they were retired. reap_ready frees
// what is safe whenever the device's online service is not running (the drain is then bounded
// by the calls in flight), and growth is geometric (x1.5), so a sequence of growing calls
// retires O(log n) blocks, not one per call. reap_retired (mv_destroy,
// mv_set_committee: the service stopped) frees the rest.
struct Retired {
  int device;
  void* p;
  bool host;
  hipEvent_t guard;
};
std::mutex g_retired_mu;
std::vector<Retired> g_retired;
std::atomic<int> g_retired_n{0};

void retire(void* p, bool host, hipEvent_t guard) {
  int d = 0;
  (void)hipGetDevice(&d);
  std::lock_guard<std::mutex> lk(g_retired_mu);
  g_retired.push_back(Retired{d, p, host, guard});
  g_retired_n.store((int)g_retired.size());
}

// Frees the retired blocks of `device` (its current device must be set; drains the device).
void reap_retired(int device) {
  std::vector<Retired> mine;
  {
    std::lock_guard<std::mutex> lk(g_retired_mu);
    auto it = std::stable_partition(g_retired.begin(), g_retired.end(),
                                    [device](const Retired& r) { return r.device != device; });
    mine.assign(it, g_retired.end());
    g_retired.erase(it, g_retired.end());
    g_retired_n.store((int)g_retired.size());
  }
  for (const Retired& r : mine) (void)(r.host ? hipHostFree(r.p) : hipFree(r.p));
}

// Frees the retired blocks of `device` that no call in flight can read (guard complete or
// none); the caller has checked that no resident kernel runs on the device.
void reap_ready(int device) {
  if (g_retired_n.load(std::memory_order_relaxed) == 0) return;
  std::vector<Retired> done;
  {
    std::lock_guard<std::mutex> lk(g_retired_mu);
    auto it = std::stable_partition(g_retired.begin(), g_retired.end(), [device](const Retired& r) {
      if (r.device != device) return true;
      if (!r.guard) return false;
      const hipError_t q = hipEventQuery(r.guard);
      if (q != hipSuccess) (void)hipGetLastError();  // hipErrorNotReady: still in use
      return q != hipSuccess;
    });
    done.assign(it, g_retired.end());
    g_retired.erase(it, g_retired.end());
    g_retired_n.store((int)g_retired.size());
  }
  for (const Retired& r : done) (void)(r.host ? hipHostFree(r.p) : hipFree(r.p));
}

// the size to allocate for `bytes` when `cap` is too small: x1.5 steps, exact on first use
size_t grown(size_t cap, size_t bytes) { return std::max<size_t>({bytes, 4096, cap ? cap + cap / 2 : 0}); }

struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  // guard: the completion event of the calls that used the buffer (see Retired), or null
  hipError_t ensure(size_t bytes, hipEvent_t guard = nullptr) {
    if (bytes <= cap) return hipSuccess;
    const size_t want = grown(cap, bytes);
    if (p) retire(p, false, guard);
    p = nullptr;
    cap = 0;
    hipError_t e = hipMalloc(&p, want);
    if (e != hipSuccess && want > bytes) {  // the geometric step does not fit: exactly
      (void)hipGetLastError();
      e = hipMalloc(&p, std::max<size_t>(bytes, 4096));
      if (e == hipSuccess) cap = std::max<size_t>(bytes, 4096);
      return e;
    }
    if (e == hipSuccess) cap = want;
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
  template <class T>
  T* as() const {
    return static_cast<T*>(p);
  }
};

struct HostBuf {
  void* p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t bytes) {
    if (bytes <= cap) return hipSuccess;
    const size_t want = grown(cap, bytes);
    if (p) retire(p, true, nullptr);  // pinned staging: host-buffer calls only (synchronous)
    p = nullptr;
    cap = 0;
    hipError_t e = hipHostMalloc(&p, want, hipHostMallocDefault);
    if (e != hipSuccess && want > bytes) {
      (void)hipGetLastError();
      e = hipHostMalloc(&p, std::max<size_t>(bytes, 4096), hipHostMallocDefault);
      if (e == hipSuccess) cap = std::max<size_t>(bytes, 4096);
      return e;
    }
    if (e == hipSuccess) cap = want;
    return e;
  }
  void release() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
  }
  template <class T>
  T* as() const {
    return static_cast<T*>(p);
  }
};

struct OnlineSvc;

struct Device {
  int id = 0;
  hipStream_t stream = nullptr;
  // host-buffer batch verifies: two compute streams and double-buffered device inputs, so
  // the (pageable) H2D of one chunk runs beside the previous chunk's verification
  hipStream_t pstream[2] = {nullptr, nullptr};
  // (three input buffer sets: the streamed pinned path's batches rotate over them; four measured
  // the same for two concurrent callers, profiles/r06/e2e_two_callers.txt)
  static constexpr int kPinBufs = 3;
  DevBuf pin_msg[kPinBufs], pin_sig[kPinBufs], pin_pk[kPinBufs], pin_st[kPinBufs];
  hipEvent_t pin_free[kPinBufs] = {};
  // pinned inputs: per-chunk "copied" events of the input buffers (verify_host_streamed)
  static constexpr int kMaxChunks = 64;
  hipEvent_t chunk_ev[kPinBufs][kMaxChunks] = {};
  int pin_next = 0;  // the next batch's input buffer and compute stream (rotating across calls)
  // Pinned signature calls in flight (verify_host_streamed): each holds one of kSigCalls status
  // staging slots from its enqueue until its verdicts are copied out; the enqueue runs under
  // ctx->mu, the wait does not, so one caller's copies run beside another's verification.
  static constexpr int kSigCalls = 4;
  HostBuf sig_stage[kSigCalls];
  hipEvent_t sig_done[kSigCalls][2] = {};
  bool sig_busy[kSigCalls] = {};
  // the batch path's preparation chain (MV_PREP_CHAIN): recorded after each batch's k_bv_prep;
  // the next batch's k_bv_prep waits for it (prep_chained: recorded at least once)
  hipEvent_t prep_chain = nullptr;
  bool prep_chained = false;
  DevBuf btab, combB, scratch, msg, sig, pk, keyidx, status, bytes, off, len, out2;
  // committee: key encodings, stakes, per-key comb tables C_A, per-key decode flags
  DevBuf committee_pk, stakes, combA, keyok;
  // scratch rings: consecutive calls rotate over kSlots slots, so a call on one stream can
  // run while the previous ones (on other streams) finish their latency-bound tails; an
  // event per slot orders reuse across streams. Batch path: bscr/vscr; blocks: blk.
#ifndef MV_SLOTS
#define MV_SLOTS 3
#endif
  static constexpr int kSlots = MV_SLOTS;
  static constexpr int kFlagWords = 1 + mvk::BATCH_MAX_GROUPS;
  DevBuf bscr[kSlots], vscr[kSlots];
  hipEvent_t slot_done[kSlots] = {};
  bool slot_used[kSlots] = {};
  int next_slot = 0;
  // the single-path batches' rejected-signature counts, one device word per flag-ring entry
  DevBuf rejects;
  // the batch flags of each call, copied to pinned host words behind it, in a ring larger
  // than the scratch ring: read (without blocking) once flag_ev has completed;
  // flag_groups[e] groups pending. A call blocks the host only with kFlagRing calls in flight.
  static constexpr int kFlagRing = 16;
  uint32_t* h_flags = nullptr;  // kFlagRing x kFlagWords, pinned
  uint32_t flag_groups[kFlagRing] = {};
  hipEvent_t flag_ev[kFlagRing] = {};
  int flag_next = 0;
  // single-verify scratch (k_verify's per-wave tables), same ring
  DevBuf sscr[kSlots];
  hipEvent_t sscr_done[kSlots] = {};
  bool sscr_used[kSlots] = {};
  int sscr_next = 0;
  // device-API block-pipeline scratch: a ring of two slots (a caller alternating two streams
  // keeps one call running beside the next), all grown together on first use so no slot is
  // allocated inside a caller's steady state (a 2^21-block slot is ~21 GB; round 3's four
  // lazily grown slots put one ~0.8 s allocation into the driver's timed steps)
#ifndef MV_BLK_SLOTS
#define MV_BLK_SLOTS 3
#endif
  static constexpr int kBlkSlots = MV_BLK_SLOTS;
  DevBuf blk[kBlkSlots];
  hipEvent_t blk_done[kBlkSlots] = {};
  bool blk_used[kBlkSlots] = {};
  int blk_next = 0;
  // batch-size block calls: the second half's parse on an aux stream beside the first half's
  // hash (enqueue_blocks). One aux stream and event pair per scratch owner (ring slot or pass
  // set), so two calls in flight never queue their second halves behind each other.
  struct BlkAux {
    hipStream_t stream = nullptr;
    hipEvent_t ev[2] = {};
  };
  BlkAux blk_aux[kBlkSlots];
  HostBuf h_in, h_out;
  // mv_verify_blocks passes (the submission queue): kPassSets sets of pinned staging, device
  // buffers and a stream each, so pass k + 1 is packed and enqueued while passes k, k - 1, ...
  // run (an online pass is a few workgroups: passes on distinct hardware queues run side by side)
  static constexpr int kPassSets = 4;
  hipStream_t qstream[kPassSets] = {};  // one per pass set
  struct PassSet {
    HostBuf h_in, h_out;
    DevBuf bytes, out2, scr;  // scr: the block pipeline's scratch for this set's passes
    BlkAux aux;               // the two-halves parse of a large host-fed chunk
    hipStream_t stream = nullptr;  // qstream[k]
    hipEvent_t done = nullptr;
    // the chunk in flight: items [lo, lo + m) of `it`, outputs in h_out when finished
    const void* it = nullptr;
    uint64_t lo = 0;
    uint32_t m = 0;
    bool inflight = false;
  };
  PassSet pset[kPassSets];
  bool committee_loaded = false;
  // WAL replay (wal.hip): crc tables, walk records, per-map counts / flags / offsets, entries,
  // the image and outputs of host-buffer calls
  DevBuf wal_tab, wal_rec, wal_mcount, wal_mflag, wal_moff, wal_ent, wal_ff, wal_img, wal_pos, wal_tag, wal_len,
      wal_st;
  int cus = 0;
  // the resident online service (k_online) of this device, made on first use
  std::shared_ptr<OnlineSvc> online;
};

struct PendingEvents {
  int device;
  int first_stage;  // stage index of events[0] -> events[1]
  std::vector<hipEvent_t> events;
};

}  // namespace

struct mv_ctx {
  std::mutex mu;
  std::vector<Device> devs;
  std::string err;
  uint32_t max_batch = 1u << 20;
  uint32_t flags = 0;
  uint32_t secret[8] = {0};         // batch-path z_i PRF key (from /dev/urandom)
  std::atomic<uint64_t> calls{0};   // batch calls, the PRF's per-call input
  std::atomic<uint64_t> batches{0}, fallbacks{0}, groups_run{0}, groups_failed{0};
  // sub-batch equations per batch: groups_fixed != 0 forces that many; 0 = adaptive:
  // base_groups equations (one: every group adds 16 x 2^15 buckets to the bucket and reduce
  // kernels; config 2 measured 267 M/s at one group against 241 M/s at four), and after a
  // batch whose equation failed, the next kGuardBatches batches are cut into guard_groups
  // (a failure then re-verifies 1/8 of the batch).
  uint32_t groups_fixed = 0;
  uint32_t base_groups = 1;
  uint32_t guard_groups = 8;
  std::atomic<int> guard_left{0};
  // batches still to send straight to the single path (dense failures, kSingleRun), and the
  // counts of batches by route
  std::atomic<int> single_left{0};
  std::atomic<uint64_t> single_batches{0}, dense_failures{0};
  // stage timing (mv_set_stage_timing): event sets of calls not yet read back
  bool stage_timing = false;
  std::mutex tmu;
  std::vector<PendingEvents> pending;
  double stage_ms[MV_NSTAGES] = {0};
  uint64_t stage_calls[MV_NSTAGES] = {0};
  std::atomic<bool> has_committee{false};
  std::condition_variable sig_cv;  // a pinned signature call released its staging slot (Device::sig_busy)
  mvh::Committee committee;
  // block submission queue (mv_verify_blocks): concurrent callers' requests are merged into
  // one device pass by whichever caller finds the engine idle (flat combining)
  struct BlockReq;
  std::mutex q_mu;
  std::condition_variable q_cv;
  std::deque<BlockReq*> q;
  bool q_packing = false;                // a combining caller is packing / enqueueing a pass
  bool q_set_busy[Device::kPassSets] = {};  // pass sets with a pass in flight
  int q_sets = 0;                          // pass sets in use (MV_PASS_SETS, default kPassSets)
  // linger (MV_Q_LINGER_US): a combining caller that finds fewer requests queued than the last
  // finished pass carried waits briefly for the rest of that pass's callers to come back
  std::condition_variable q_linger_cv;
  bool q_lingering = false;
  size_t q_last_calls = 0;
  std::atomic<uint64_t> q_calls{0}, q_passes{0};
  // online requests hold it shared for their whole life; mv_set_committee and mv_destroy take it
  // exclusively (the resident kernel reads the committee's tables)
  std::shared_mutex com_mu;
  std::atomic<uint64_t> online_rr{0};
  std::vector<size_t> online_devs;  // devs[] index of the first logical shard of each GPU
  // the runtime switches, read from the environment at mv_create (knobs_from_env) and changed
  // only by mv_set_option (diagnostics, between calls)
  mvk::Knobs kn;
};

struct mv_ctx::BlockReq {
  const uint8_t* buf;
  const uint64_t *off, *len;
  uint32_t n;
  uint8_t *status, *md, *bd;
  mv_status rc = MV_OK;
  std::string err;
  bool taken = false;             // in a pass (q_mu)
  std::atomic<bool> done{false};  // verdicts delivered (set under q_mu, may be polled without it)
};

namespace {

// Errors are recorded in the calling thread's slot (shard threads of one call each own
// one) and published to ctx->err by the thread that returns to the caller.
thread_local std::string* t_err = nullptr;

void record_err(mv_ctx* ctx, const std::string& msg) {
  if (t_err) *t_err = msg;
  else if (ctx) ctx->err = msg;
}

#define HIPCHK(ctx, expr)                                                                          \
  do {                                                                                             \
    hipError_t e_ = (expr);                                                                        \
    if (e_ != hipSuccess) {                                                                        \
      record_err((ctx), std::string(#expr) + ": " + hipGetErrorString(e_));                        \
      return MV_E_HIP;                                                                             \
    }                                                                                              \
  } while (0)

// HIPCHK for functions that carry the status in `rc` (the first error is kept, no early return)
#define HIPCHK_RC(ctx, rc, expr)                                                  \
  do {                                                                            \
    hipError_t e_ = (expr);                                                       \
    if (e_ != hipSuccess && (rc) == MV_OK) {                                      \
      record_err((ctx), std::string(#expr) + ": " + hipGetErrorString(e_));       \
      (rc) = MV_E_HIP;                                                            \
    }                                                                             \
  } while (0)

mv_status set_err(mv_ctx* ctx, mv_status code, const std::string& msg) {
  record_err(ctx, msg);
  return code;
}

// Runs fn(device, cut[d], cut[d + 1]) for every device with a non-empty shard, one thread
// per device (cut: nd + 1 ascending item indices from 0 to n).
template <class Fn>
mv_status for_each_cut(mv_ctx* ctx, const std::vector<uint64_t>& cut, Fn fn) {
  const size_t nd = ctx->devs.size();
  std::vector<mv_status> rc(nd, MV_OK);
  std::vector<std::string> errs(nd);
  std::vector<std::thread> th;
  for (size_t d = 0; d < nd; d++) {
    const uint64_t lo = cut[d], hi = cut[d + 1];
    if (lo == hi) continue;
    th.emplace_back([&, d, lo, hi] {
      t_err = &errs[d];
      rc[d] = fn(ctx->devs[d], lo, hi);
      t_err = nullptr;
    });
  }
  for (auto& t : th) t.join();
  for (size_t d = 0; d < nd; d++)
    if (rc[d] != MV_OK) {
      ctx->err = errs[d];
      return rc[d];
    }
  return MV_OK;
}

// Runs fn(device, lo, hi) for each device's contiguous shard of [0, n) (equal counts).
template <class Fn>
mv_status for_each_shard(mv_ctx* ctx, uint64_t n, Fn fn) {
  const size_t nd = ctx->devs.size();
  if (nd == 1 || n < 2 * 256) return fn(ctx->devs[0], 0, n);
  std::vector<uint64_t> cut(nd + 1);
  for (size_t d = 0; d <= nd; d++) cut[d] = n * d / nd;
  return for_each_cut(ctx, cut, fn);
}

// count + 1 timing events (empty when stage timing is off)
mv_status make_events(mv_ctx* ctx, int count, std::vector<hipEvent_t>& evs) {
  evs.clear();
  if (!ctx->stage_timing) return MV_OK;
  evs.assign(count + 1, nullptr);
  for (auto& ev : evs) HIPCHK(ctx, hipEventCreate(&ev));
  return MV_OK;
}
void keep_events(mv_ctx* ctx, int device, int first_stage, std::vector<hipEvent_t>& evs) {
  if (evs.empty()) return;
  std::lock_guard<std::mutex> lk(ctx->tmu);
  ctx->pending.push_back(PendingEvents{device, first_stage, std::move(evs)});
}

// Accounts the batch flags of every slot whose last call has completed (non-blocking):
// counters, and the adaptive group policy (a failed equation arms the guard).
void poll_flags(mv_ctx* ctx, Device& dev) {
  for (int k = 0; k < Device::kFlagRing; k++) {
    const uint32_t ng = dev.flag_groups[k];
    if (!ng) continue;
    if (hipEventQuery(dev.flag_ev[k]) != hipSuccess) {
      (void)hipGetLastError();  // hipErrorNotReady: still running
      continue;
    }
    dev.flag_groups[k] = 0;
    const uint32_t* f = dev.h_flags + k * Device::kFlagWords;
    if (ng == kSingleMark) {  // a single-path batch: f[0] = its rejected signatures
      if (f[0] >= kDenseRejects) {
        ctx->single_left.store(kSingleRun);
      } else {
        ctx->single_left.store(0);
        ctx->guard_left = kGuardBatches;  // back to the equation, guarded
      }
      continue;
    }
    ctx->batches++;
    ctx->groups_run += ng;
    uint32_t bad = 0;
    for (uint32_t g = 0; g < ng; g++) bad += f[1 + g] ? 0u : 1u;
    ctx->groups_failed += bad;
    if (!f[0]) {
      ctx->fallbacks++;
      ctx->guard_left = kGuardBatches;
      if (ng >= 2 && 2 * bad >= ng && ctx->groups_fixed == 0) {  // dense: the MSM was wasted
        ctx->dense_failures++;
        ctx->single_left.store(kSingleRun);
      }
    }
  }
}

uint32_t pick_groups(mv_ctx* ctx) {
  if (ctx->groups_fixed) return ctx->groups_fixed;
  if (ctx->guard_left.fetch_sub(1) > 0) return ctx->guard_groups;
  ctx->guard_left.store(0);
  return ctx->base_groups;
}

mv_status enqueue_verify(mv_ctx* ctx, Device& dev, const uint8_t* d_msg, const uint8_t* d_sig, const uint8_t* d_pk,
                         const uint32_t* d_key_idx, uint32_t n, uint8_t* d_status, hipStream_t s);
mv_status enqueue_committee_verify(mv_ctx* ctx, Device& dev, const uint8_t* d_msg, const uint8_t* d_sig,
                                   const uint32_t* d_kidx, uint32_t n, uint8_t* d_status, hipStream_t s,
                                   const mvk::BlockVerdictOut* bv = nullptr, const mvk::BlockHashIn* hin = nullptr,
                                   const mvk::BlockIngestIn* ing = nullptr);

// Enqueues the batch path (batch.hip) for n signatures on stream s. flag_dst (optional,
// device) receives the all-groups flag word.
mv_status enqueue_batch(mv_ctx* ctx, Device& dev, const uint8_t* d_msg, const uint8_t* d_sig, const uint8_t* d_pk,
                        const uint32_t* d_key_idx, uint32_t n, uint8_t* d_status, hipStream_t s,
                        uint32_t* flag_dst, const mvk::ChunkGate* gate = nullptr, bool caller_stream = false) {
  poll_flags(ctx, dev);
  const int slot = dev.next_slot;
  dev.next_slot = (slot + 1) % Device::kSlots;
  if (!dev.slot_done[slot]) HIPCHK(ctx, hipEventCreateWithFlags(&dev.slot_done[slot], hipEventDisableTiming));
  if (!dev.h_flags) {
    HIPCHK(ctx, hipHostMalloc((void**)&dev.h_flags, sizeof(uint32_t) * Device::kFlagRing * Device::kFlagWords,
                              hipHostMallocDefault));
    memset(dev.h_flags, 0, sizeof(uint32_t) * Device::kFlagRing * Device::kFlagWords);
  }
  const int fe = dev.flag_next;
  dev.flag_next = (fe + 1) % Device::kFlagRing;
  if (!dev.flag_ev[fe]) HIPCHK(ctx, hipEventCreateWithFlags(&dev.flag_ev[fe], hipEventDisableTiming));
  if (dev.flag_groups[fe]) {  // kFlagRing calls in flight: the oldest must be accounted before its words are reused
    HIPCHK(ctx, hipEventSynchronize(dev.flag_ev[fe]));
    poll_flags(ctx, dev);
  }
  const bool com_a = d_key_idx && dev.committee_loaded && d_pk == dev.committee_pk.as<uint8_t>() &&
                     !(ctx->flags & MV_FLAG_NO_COMB);
  if (ctx->groups_fixed == 0 && ctx->single_left.load() > 0) {
    // dense failures (kSingleRun): every signature verified alone, no combined equation; the
    // rejected count decides whether the next batches try the equation again (poll_flags)
    ctx->single_left--;
    dev.next_slot = slot;  // no batch scratch used
    if (gate && gate->n)
      for (uint32_t c = 0; c < gate->n; c++) HIPCHK(ctx, hipStreamWaitEvent(s, gate->ready[c], 0));
    mv_status st = com_a ? enqueue_committee_verify(ctx, dev, d_msg, d_sig, d_key_idx, n, d_status, s)
                         : enqueue_verify(ctx, dev, d_msg, d_sig, d_pk, d_key_idx, n, d_status, s);
    if (st != MV_OK) return st;
    HIPCHK(ctx, dev.rejects.ensure(sizeof(uint32_t) * Device::kFlagRing));
    uint32_t* cnt = dev.rejects.as<uint32_t>() + fe;
    HIPCHK(ctx, mvk::launch_count_rejects(d_status, n, cnt, s));
    if (flag_dst) HIPCHK(ctx, hipMemsetAsync(flag_dst, 0, 4, s));  // no combination was checked
    HIPCHK(ctx, hipMemcpyAsync(dev.h_flags + fe * Device::kFlagWords, cnt, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    HIPCHK(ctx, hipEventRecord(dev.flag_ev[fe], s));
    dev.flag_groups[fe] = kSingleMark;
    ctx->single_batches++;
    return MV_OK;
  }
  if (dev.slot_used[slot]) HIPCHK(ctx, hipStreamWaitEvent(s, dev.slot_done[slot], 0));  // device-side order only
  const uint32_t groups = pick_groups(ctx);
  // scratch for the largest group count, so the adaptive policy never reallocates
  HIPCHK(ctx, dev.bscr[slot].ensure(mvk::batch_scratch_bytes(n, mvk::BATCH_MAX_GROUPS), dev.slot_done[slot]));
  HIPCHK(ctx, dev.vscr[slot].ensure(mvk::verify_scratch_bytes(n), dev.slot_done[slot]));
  uint32_t key[10];
  memcpy(key, ctx->secret, 32);
  const uint64_t call = ctx->calls.fetch_add(1);
  key[8] = (uint32_t)call;
  key[9] = (uint32_t)(call >> 32);
  uint32_t* flag = nullptr;
  std::vector<hipEvent_t> evs;
  mv_status st = make_events(ctx, mvk::BATCH_STAGES, evs);
  if (st != MV_OK) return st;
  // committee keys (com_a): A comes from the comb tables built at mv_set_committee (no
  // per-signature decode)
  hipEvent_t chain[2] = {};
  // on a caller's stream only when asked (MV_PREP_CHAIN=2): the chain orders the caller's streams
  // behind each other's preparations, which the caller may not expect (its own gates could then
  // deadlock them)
  const bool chained = ctx->kn.prep_chain && !(gate && gate->n) && (!caller_stream || ctx->kn.prep_chain >= 2);
  if (chained) {
    if (!dev.prep_chain) HIPCHK(ctx, hipEventCreateWithFlags(&dev.prep_chain, hipEventDisableTiming));
    chain[0] = dev.prep_chained ? dev.prep_chain : nullptr;
    chain[1] = dev.prep_chain;
  }
  HIPCHK(ctx, mvk::launch_verify_batch(ctx->kn, d_msg, d_sig, d_pk, d_key_idx, n, groups, key, dev.btab.p, dev.bscr[slot].p,
                                       dev.vscr[slot].p, d_status, s, &flag, evs.empty() ? nullptr : evs.data(),
                                       com_a ? dev.combA.p : nullptr, com_a ? dev.keyok.as<uint8_t>() : nullptr,
                                       com_a ? (uint32_t)ctx->committee.size() : 0u, dev.combB.p, gate,
                                       chained ? chain : nullptr));
  if (chained) dev.prep_chained = true;
  keep_events(ctx, dev.id, 0, evs);
  if (flag_dst) HIPCHK(ctx, hipMemcpyAsync(flag_dst, flag, 4, hipMemcpyDeviceToDevice, s));
  const uint32_t ng = (n + mvk::batch_group_size(n, groups) - 1) / mvk::batch_group_size(n, groups);
  HIPCHK(ctx, hipMemcpyAsync(dev.h_flags + fe * Device::kFlagWords, flag, sizeof(uint32_t) * (1 + ng),
                             hipMemcpyDeviceToHost, s));
  HIPCHK(ctx, hipEventRecord(dev.slot_done[slot], s));
  HIPCHK(ctx, hipEventRecord(dev.flag_ev[fe], s));
  dev.slot_used[slot] = true;
  dev.flag_groups[fe] = ng;
  return MV_OK;
}

// k_verify (single path) on stream s with the device's scratch ring (per-wave tables)
mv_status enqueue_verify(mv_ctx* ctx, Device& dev, const uint8_t* d_msg, const uint8_t* d_sig, const uint8_t* d_pk,
                         const uint32_t* d_key_idx, uint32_t n, uint8_t* d_status, hipStream_t s) {
  if (n == 0) return MV_OK;
  const int slot = dev.sscr_next;
  dev.sscr_next = (slot + 1) % Device::kSlots;
  if (!dev.sscr_done[slot]) HIPCHK(ctx, hipEventCreateWithFlags(&dev.sscr_done[slot], hipEventDisableTiming));
  if (dev.sscr_used[slot]) HIPCHK(ctx, hipStreamWaitEvent(s, dev.sscr_done[slot], 0));
  // (growth retires the old buffer, which another stream's call may still read: no drain)
  HIPCHK(ctx, dev.sscr[slot].ensure(mvk::verify_scratch_bytes(n), dev.sscr_done[slot]));
  HIPCHK(ctx, mvk::launch_verify(ctx->kn, d_msg, d_sig, d_pk, d_key_idx, n, dev.btab.p, dev.sscr[slot].p, d_status, s));
  HIPCHK(ctx, hipEventRecord(dev.sscr_done[slot], s));
  dev.sscr_used[slot] = true;
  return MV_OK;
}

// Committee-key signatures one by one: comb tables (comb.hip) or, with MV_FLAG_NO_COMB,
// the per-signature ladder (k_verify).
// bv: the block verdict fused into the comb kernel (the block path); null otherwise.
mv_status enqueue_committee_verify(mv_ctx* ctx, Device& dev, const uint8_t* d_msg, const uint8_t* d_sig,
                                   const uint32_t* d_kidx, uint32_t n, uint8_t* d_status, hipStream_t s,
                                   const mvk::BlockVerdictOut* bv, const mvk::BlockHashIn* hin,
                                   const mvk::BlockIngestIn* ing) {
  if (!(ctx->flags & MV_FLAG_NO_COMB)) {
    HIPCHK(ctx, mvk::launch_verify_comb(ctx->kn, d_msg, d_sig, dev.committee_pk.as<uint8_t>(), d_kidx, n, dev.combB.p,
                                        dev.combA.p, dev.keyok.as<uint8_t>(), d_status, s, bv, hin, ing));
  } else {
    return enqueue_verify(ctx, dev, d_msg, d_sig, dev.committee_pk.as<uint8_t>(), d_kidx, n, d_status, s);
  }
  return MV_OK;
}

// The device block pipeline on stream s (enqueue only): batch-size calls k_block_walk (parse,
// checks and both digests in one pass over the bincode) -> k_block_digest_gate -> batch path
// -> k_block_verdict; smaller calls the committee comb kernels (which parse and hash their own
// blocks on the online path; k_block_ingest -> k_hash_comb_pre -> k_comb_post for small
// batches of long blocks). d_md / d_bd may be null (scratch then).
// own: scratch owned by the caller (a submission-queue pass set, whose reuse is ordered by its
// own completion event): no ring slot, no slot events (two runtime calls less per pass).
mv_status enqueue_blocks(mv_ctx* ctx, Device& dev, const uint8_t* d_buf, uint64_t buf_bytes, const uint64_t* d_off,
                         const uint64_t* d_len, uint32_t n, uint8_t* d_status, uint8_t* d_md, uint8_t* d_bd,
                         hipStream_t s, DevBuf* own = nullptr, Device::BlkAux* own_aux = nullptr) {
  if (n == 0) return MV_OK;
  const mvh::Committee& com = ctx->committee;
  int slot = -1;
  if (!own) {
    slot = dev.blk_next;
    dev.blk_next = (slot + 1) % Device::kBlkSlots;
    if (!dev.blk_done[slot]) HIPCHK(ctx, hipEventCreateWithFlags(&dev.blk_done[slot], hipEventDisableTiming));
    if (dev.blk_used[slot]) {
      // skip the cross-stream wait when the slot's previous pass has finished (the common case
      // on the online path, where a wait costs a queue drain)
      const hipError_t q = hipEventQuery(dev.blk_done[slot]);
      if (q != hipSuccess) {
        (void)hipGetLastError();  // hipErrorNotReady is not an error here
        HIPCHK(ctx, hipStreamWaitEvent(s, dev.blk_done[slot], 0));
      }
    }
  }
  DevBuf& scr = own ? *own : dev.blk[slot];
  // small batches of long blocks: the comb verify's signature-only half beside the hash
  // bytes per block from which the split pays (MV_COMB_SPLIT_BYTES: tests and experiments; 0 = never)
  const uint64_t split_bytes = (uint64_t)std::max<int64_t>(0, ctx->kn.comb_split_bytes);
  const bool batch = !(ctx->flags & MV_FLAG_NO_BATCH) && n >= MV_BATCH_MIN;
  const bool split = !batch && !(ctx->flags & MV_FLAG_NO_COMB) && split_bytes && buf_bytes >= split_bytes * (uint64_t)n;
  // scratch: stage | pre_off | pre_len | sig | key_idx | facts | claimed | sig status | md | bd
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  const size_t nn = n;
  size_t o = 0;
  const size_t o_stage = o;
  // Batch-size calls (MV_BLK_WALK=1, default): k_block_walk reads each block's bincode once and
  // writes only the per-block outputs, so no P || sig is staged (18.9 GB of HBM
  // traffic less per 2^20 config-4 blocks, and no stage buffer). MV_BLK_WALK=0: the staged form
  // (k_block_ingest stages P || sig, k_b2_lane hashes it); small calls always stage.
  const bool walk = batch && !split && ctx->kn.blk_walk && com.size() <= 512;
  const bool need_stage = !walk;
  o += need_stage ? al(buf_bytes + 256) : al(256);
  const size_t o_poff = o;
  o += al(8 * nn);
  const size_t o_plen = o;
  o += al(8 * nn);
  const size_t o_sig = o;
  o += al(64 * nn);
  const size_t o_kidx = o;
  o += al(4 * nn);
  const size_t o_facts = o;
  o += al(4 * nn);
  const size_t o_claim = o;
  o += al(32 * nn);
  const size_t o_sst = o;
  o += al(nn);
  const size_t o_md = o;
  o += al(32 * nn);
  const size_t o_bd = o;
  o += al(32 * nn);
  const size_t o_q = o;
  if (split) o += 2 * al(144 * nn) + al(nn);
  if (!own && scr.cap < o) {
    // grow every ring slot at once, so the ring never allocates again at this size (the old
    // buffers are retired, not freed: another stream's call may still read them; no drain)
    for (int k = 0; k < Device::kBlkSlots; k++) HIPCHK(ctx, dev.blk[k].ensure(o, dev.blk_done[k]));
  }
  HIPCHK(ctx, scr.ensure(o, own ? nullptr : dev.blk_done[slot]));
  char* b = scr.as<char>();
  uint8_t* stage = (uint8_t*)(b + o_stage);
  uint64_t* poff = (uint64_t*)(b + o_poff);
  uint64_t* plen = (uint64_t*)(b + o_plen);
  uint8_t* sig = (uint8_t*)(b + o_sig);
  uint32_t* kidx = (uint32_t*)(b + o_kidx);
  uint32_t* facts = (uint32_t*)(b + o_facts);
  uint8_t* claimed = (uint8_t*)(b + o_claim);
  uint8_t* sst = (uint8_t*)(b + o_sst);
  uint8_t* md = d_md ? d_md : (uint8_t*)(b + o_md);
  uint8_t* bd = d_bd ? d_bd : (uint8_t*)(b + o_bd);
  std::vector<hipEvent_t> evs;
  mv_status st = make_events(ctx, kBlockStages, evs);
  if (st != MV_OK) return st;
  auto mark = [&](int i) -> hipError_t { return evs.empty() ? hipSuccess : hipEventRecord(evs[i], s); };
  HIPCHK(ctx, mark(0));
  uint8_t* rbuf = (uint8_t*)(b + o_q);
  uint8_t* sbuf = rbuf + al(144 * nn);
  uint8_t* qflags = sbuf + al(144 * nn);
  // short blocks on the online path: the digests are computed inside the committee verify
  // (k_verify_comb16's A wave hashes its blocks before the challenge), one launch less
  // (MV_HASH_IN_COMB=0, A/B: a separate hash launch)
  const bool hash_in_comb = !split && !batch && !(ctx->flags & MV_FLAG_NO_COMB) &&
                            mvk::comb_short_chain(ctx->kn, n) && ctx->kn.hash_in_comb;
  const mvk::BlockHashIn hin{stage, poff, plen, md, bd};
  // ... and the parse too: k_verify_comb16 ingests its own blocks (one wave per block), so an
  // online pass is one kernel launch (MV_INGEST_IN_COMB=0: a separate k_block_ingest, A/B)
  const bool ingest_in_comb = hash_in_comb && ctx->kn.ingest_in_comb;
  const mvk::BlockIngestIn ing{d_buf, d_off, d_len, dev.stakes.as<uint64_t>(), com.size(), com.epoch,
                               com.quorum_threshold, stage, poff, plen, sig, kidx, facts, claimed};
  if (ingest_in_comb) {
    HIPCHK(ctx, mark(1));
  } else if (walk) {
    HIPCHK(ctx, mvk::launch_block_walk(d_buf, d_off, d_len, n, dev.stakes.as<uint64_t>(), com.size(), com.epoch,
                                       com.quorum_threshold, sig, kidx, facts, claimed, md, bd, s));
    HIPCHK(ctx, mark(1));
  } else if (batch && !split && !ctx->stage_timing && n >= 2 * MV_BATCH_MIN + 64 && ctx->kn.blk_pipe && (!own || own_aux)) {
    // Batch-size calls, two halves: the HBM-bound parse of the second half runs on another
    // stream beside the VALU-bound hash of the first (the two streams of a caller's
    // alternating calls otherwise start in phase, parse beside parse). MV_BLK_PIPE=0: one
    // stream. Not under stage timing, whose per-stage events need the stages in sequence.
    // both halves >= MV_BATCH_MIN, so both hash on the batch-size kernel (n >= 2 MV_BATCH_MIN + 64)
    const uint32_t h = ((n / 2) + 63) & ~63u;
    Device::BlkAux& ax = own ? *own_aux : dev.blk_aux[slot];
    if (!ax.stream) HIPCHK(ctx, hipStreamCreateWithFlags(&ax.stream, hipStreamNonBlocking));
    for (int k = 0; k < 2; k++)
      if (!ax.ev[k]) HIPCHK(ctx, hipEventCreateWithFlags(&ax.ev[k], hipEventDisableTiming));
    hipStream_t aux = ax.stream;
    auto parse = [&](uint32_t lo, uint32_t hi, hipStream_t st) {
      return mvk::launch_block_parse(ctx->kn, d_buf, d_off + lo, d_len + lo, hi - lo, dev.stakes.as<uint64_t>(), com.size(),
                                     com.epoch, com.quorum_threshold, stage, poff + lo, plen + lo, sig + 64 * (size_t)lo,
                                     kidx + lo, facts + lo, claimed + 32 * (size_t)lo, st);
    };
    auto hash = [&](uint32_t lo, uint32_t hi) {
      return mvk::launch_block_hash(ctx->kn, stage, poff + lo, plen + lo, hi - lo, md + 32 * (size_t)lo,
                                    bd + 32 * (size_t)lo, s);
    };
    HIPCHK(ctx, parse(0, h, s));
    HIPCHK(ctx, hipEventRecord(ax.ev[0], s));
    HIPCHK(ctx, hipStreamWaitEvent(aux, ax.ev[0], 0));
    HIPCHK(ctx, parse(h, n, aux));
    HIPCHK(ctx, hipEventRecord(ax.ev[1], aux));
    HIPCHK(ctx, mark(1));
    HIPCHK(ctx, hash(0, h));
    HIPCHK(ctx, hipStreamWaitEvent(s, ax.ev[1], 0));
    HIPCHK(ctx, hash(h, n));
  } else {
    HIPCHK(ctx, mvk::launch_block_parse(ctx->kn, d_buf, d_off, d_len, n, dev.stakes.as<uint64_t>(), com.size(), com.epoch,
                                        com.quorum_threshold, stage, poff, plen, sig, kidx, facts, claimed, s));
    HIPCHK(ctx, mark(1));
    if (split)  // the hash, and beside it on workgroups of their own the signature-only terms
      HIPCHK(ctx, mvk::launch_hash_comb_pre(stage, poff, plen, n, md, bd, sig, dev.combB.p, rbuf, sbuf, qflags, s));
    else if (!hash_in_comb)
      HIPCHK(ctx, mvk::launch_block_hash(ctx->kn, stage, poff, plen, n, md, bd, s));
  }
  // a block whose digest does not match is rejected ahead of its signature (types.rs:327-332):
  // s >= l takes it out of the batch equation, so a tampered block never fails the batch (the
  // per-signature paths need no gate: the verdict puts the digest first)
  if (batch) HIPCHK(ctx, mvk::launch_block_digest_gate(claimed, bd, facts, n, sig, s));
  HIPCHK(ctx, mark(2));
  // the comb kernels write the block verdict themselves (one launch less on the online path);
  // the batch path and the MV_FLAG_NO_COMB ladder leave it to k_block_verdict
  // (MV_VERDICT_FUSED=0, A/B: the separate k_block_verdict)
  const bool fused = ctx->kn.verdict_fused && !batch && !(ctx->flags & MV_FLAG_NO_COMB);
  const mvk::BlockVerdictOut bv{facts, claimed, md, bd, d_status};
  if (batch) {
    st = enqueue_batch(ctx, dev, md, sig, dev.committee_pk.as<uint8_t>(), kidx, n, sst, s, nullptr, nullptr,
                       own == nullptr);  // own == nullptr: mv_dev_verify_blocks on the caller's stream
  } else if (split) {
    HIPCHK(ctx, mvk::launch_comb_post(md, sig, dev.committee_pk.as<uint8_t>(), kidx, n, dev.combA.p,
                                      dev.keyok.as<uint8_t>(), rbuf, sbuf, qflags, sst, s, fused ? &bv : nullptr));
  } else {
    st = enqueue_committee_verify(ctx, dev, md, sig, kidx, n, sst, s, fused ? &bv : nullptr,
                                  hash_in_comb ? &hin : nullptr, ingest_in_comb ? &ing : nullptr);
  }
  if (st != MV_OK) return st;
  HIPCHK(ctx, mark(3));
  if (!fused) HIPCHK(ctx, mvk::launch_block_verdict(facts, claimed, md, bd, sst, n, d_status, s));
  HIPCHK(ctx, mark(4));
  keep_events(ctx, dev.id, kBlockStage0, evs);
  if (!own) {
    HIPCHK(ctx, hipEventRecord(dev.blk_done[slot], s));
    dev.blk_used[slot] = true;
  }
  return MV_OK;
}

// mv_verify_blocks with MV_FLAG_HOST_PARSE: bincode parsed on the host (block_codec.cpp),
// staged pre-images to the device. Kept as the cross-check of the device ingest path.
mv_status verify_blocks_host_parse(mv_ctx* ctx, const uint8_t* buf, const uint64_t* off, const uint64_t* len,
                                   uint32_t n, uint8_t* status, uint8_t* msg_digest, uint8_t* block_digest) {
  const mvh::Committee& com = ctx->committee;
  return for_each_shard(ctx, n, [&](Device& dev, uint64_t lo, uint64_t hi) -> mv_status {
    HIPCHK(ctx, hipSetDevice(dev.id));
    uint64_t i = lo;
    std::vector<mvh::BlockFacts> facts;
    while (i < hi) {
      // chunk: <= max_batch blocks and <= 1 GiB of staged pre-images
      uint64_t j = i, bytes = 0;
      while (j < hi && j - i < ctx->max_batch && bytes < (1ull << 30)) bytes += len[j++] + 64 + 16;
      uint32_t m = (uint32_t)(j - i);
      facts.assign(m, mvh::BlockFacts());
      HIPCHK(ctx, dev.h_in.ensure(bytes + 64));
      uint8_t* st = dev.h_in.as<uint8_t>();
      std::vector<uint64_t> soff(m), slen(m);
      std::vector<uint32_t> kidx(m);
      uint64_t pos = 0;
      for (uint32_t k = 0; k < m; k++) {
        mvh::BlockFacts& f = facts[k];
        soff[k] = pos;
        // pre-image is never longer than the bincode (only fields are dropped or re-encoded)
        bool ok = mvh::parse_block(buf + off[i + k], len[i + k], &com, st + pos, len[i + k], f);
        if (!ok) f.parsed = false;
        uint64_t L = ok ? f.preimage_len : 0;
        if (ok) memcpy(st + pos + L, f.signature, 64);
        else memset(st + pos, 0, 64);
        memset(st + pos + L + 64, 0, 8);
        slen[k] = L;
        kidx[k] = (ok && f.author < com.size()) ? (uint32_t)f.author : 0u;
        pos += (L + 64 + 15) & ~7ull;
      }
      HIPCHK(ctx, dev.bytes.ensure(pos + 64));
      HIPCHK(ctx, dev.off.ensure(8 * (size_t)m));
      HIPCHK(ctx, dev.len.ensure(8 * (size_t)m));
      HIPCHK(ctx, dev.msg.ensure(32 * (size_t)m));
      HIPCHK(ctx, dev.out2.ensure(32 * (size_t)m));
      HIPCHK(ctx, dev.sig.ensure(64 * (size_t)m));
      HIPCHK(ctx, dev.keyidx.ensure(4 * (size_t)m));
      HIPCHK(ctx, dev.status.ensure(m));
      std::vector<uint8_t> sigs(64 * (size_t)m);
      for (uint32_t k = 0; k < m; k++) {
        const mvh::BlockFacts& f = facts[k];
        memcpy(&sigs[64 * (size_t)k], f.signature, 64);
        // the verdict of a block that fails a check ahead of the signature one does not
        // depend on its signature: s = 2^256 - 1 (>= l) takes it out of the batch
        // equation (rejected up front) instead of failing the whole batch
        if (!f.parsed || f.epoch != com.epoch || f.author >= com.size() || f.round == 0)
          memset(&sigs[64 * (size_t)k + 32], 0xff, 32);
      }
      HIPCHK(ctx, hipMemcpyAsync(dev.bytes.p, st, pos, hipMemcpyHostToDevice, dev.stream));
      HIPCHK(ctx, hipMemcpyAsync(dev.off.p, soff.data(), 8 * (size_t)m, hipMemcpyHostToDevice, dev.stream));
      HIPCHK(ctx, hipMemcpyAsync(dev.len.p, slen.data(), 8 * (size_t)m, hipMemcpyHostToDevice, dev.stream));
      HIPCHK(ctx, hipMemcpyAsync(dev.sig.p, sigs.data(), 64 * (size_t)m, hipMemcpyHostToDevice, dev.stream));
      HIPCHK(ctx, hipMemcpyAsync(dev.keyidx.p, kidx.data(), 4 * (size_t)m, hipMemcpyHostToDevice, dev.stream));
      // msg digests stay on the device and feed the verify kernel directly
      HIPCHK(ctx, mvk::launch_block_hash(ctx->kn, dev.bytes.as<uint8_t>(), dev.off.as<uint64_t>(), dev.len.as<uint64_t>(), m,
                                         dev.msg.as<uint8_t>(), dev.out2.as<uint8_t>(), dev.stream));
      if (!(ctx->flags & MV_FLAG_NO_BATCH) && m >= MV_BATCH_MIN) {
        mv_status st2 = enqueue_batch(ctx, dev, dev.msg.as<uint8_t>(), dev.sig.as<uint8_t>(),
                                      dev.committee_pk.as<uint8_t>(), dev.keyidx.as<uint32_t>(), m,
                                      dev.status.as<uint8_t>(), dev.stream, nullptr);
        if (st2 != MV_OK) return st2;
      } else {
        mv_status st2 = enqueue_committee_verify(ctx, dev, dev.msg.as<uint8_t>(), dev.sig.as<uint8_t>(),
                                                 dev.keyidx.as<uint32_t>(), m, dev.status.as<uint8_t>(), dev.stream);
        if (st2 != MV_OK) return st2;
      }
      std::vector<uint8_t> md(32 * (size_t)m), bd(32 * (size_t)m), ss(m);
      HIPCHK(ctx, hipMemcpyAsync(md.data(), dev.msg.p, 32 * (size_t)m, hipMemcpyDeviceToHost, dev.stream));
      HIPCHK(ctx, hipMemcpyAsync(bd.data(), dev.out2.p, 32 * (size_t)m, hipMemcpyDeviceToHost, dev.stream));
      HIPCHK(ctx, hipMemcpyAsync(ss.data(), dev.status.p, m, hipMemcpyDeviceToHost, dev.stream));
      HIPCHK(ctx, hipStreamSynchronize(dev.stream));
      poll_flags(ctx, dev);
      for (uint32_t k = 0; k < m; k++) {
        status[i + k] = mvh::block_verdict(facts[k], com, &bd[32 * (size_t)k], ss[k]);
        if (!facts[k].parsed) {  // no pre-image: zero digests, as the device path
          memset(&md[32 * (size_t)k], 0, 32);
          memset(&bd[32 * (size_t)k], 0, 32);
        }
        if (msg_digest) memcpy(msg_digest + 32 * (i + k), &md[32 * (size_t)k], 32);
        if (block_digest) memcpy(block_digest + 32 * (i + k), &bd[32 * (size_t)k], 32);
      }
      i = j;
    }
    return MV_OK;
  });
}

// cut[0..parts]: contiguous shards of [0, n) with about equal sums of weights (bytes of
// bincode for block calls): cut[d] is the item boundary whose prefix sum is
// closest to d/parts of the total; every shard is non-empty while n >= parts.
std::vector<uint64_t> balanced_cuts(const uint64_t* w, uint64_t n, uint32_t parts) {
  std::vector<long double> pre(n + 1, 0.0L);
  for (uint64_t i = 0; i < n; i++) pre[i + 1] = pre[i] + (long double)w[i];
  std::vector<uint64_t> cut(parts + 1, n);
  cut[0] = 0;
  for (uint32_t d = 1; d < parts; d++) {
    const long double target = pre[n] * d / parts;
    uint64_t c = (uint64_t)(std::lower_bound(pre.begin(), pre.end(), target) - pre.begin());
    if (c > 0 && c <= n && target - pre[c - 1] < pre[c] - target) c--;
    if (c > n) c = n;
    const uint64_t lo = cut[d - 1] + (n >= parts ? 1 : 0);
    const uint64_t hi = n >= parts ? n - (parts - d) : n;
    cut[d] = c < lo ? lo : (c > hi ? hi : c);
  }
  return cut;
}

// Device passes over lists of blocks gathered from one or several mv_verify_blocks requests.
// A chunk of blocks is packed into a pass set's pinned staging (raw bincode 8-aligned, 16 zero
// bytes after the last block, then the offset and length arrays), read by the GPU (one H2D,
// or zero-copy for small chunks), parsed, hashed and verified there, and its outputs
// [msg digests | block digests | statuses] come back to pinned memory; the verdicts are then
// scattered to each block's owner.
struct BlockItem {
  const uint8_t* p;
  uint64_t len;
  uint8_t *st, *md, *bd;
};

// packed bytes of one block (8-aligned)
inline uint64_t packed_len(const BlockItem& b) { return (b.len + 7) & ~7ull; }

// Chunk limits: <= max_batch blocks and <= MV_BLK_CHUNK_BYTES (default 256 MiB) of bincode.
// A host-fed call larger than one chunk streams: chunk c + 1 is packed, copied and enqueued
// on the other pass set while chunk c runs.
uint64_t chunk_bytes_limit(const mv_ctx* ctx) {
  return ctx->kn.blk_chunk_bytes > 0 ? (uint64_t)ctx->kn.blk_chunk_bytes : (uint64_t)(256ull << 20);
}
uint64_t chunk_end(mv_ctx* ctx, const BlockItem* it, uint64_t lo, uint64_t hi) {
  uint64_t j = lo, bytes = 0;
  const uint64_t lim = chunk_bytes_limit(ctx);
  while (j < hi && j - lo < ctx->max_batch && (bytes < lim || j == lo)) bytes += packed_len(it[j++]);
  return j;
}

// Copies items [lo, hi) into h (their packed offsets in off[], lengths in len[]), on up to
// `threads` threads for large chunks.
void pack_items(uint8_t* h, uint64_t* off, uint64_t* len, const BlockItem* it, uint64_t lo, uint64_t hi,
                size_t buf_bytes, int64_t pack_threads) {
  const uint32_t m = (uint32_t)(hi - lo);
  uint64_t pos = 0;
  for (uint32_t k = 0; k < m; k++) {
    off[k] = pos;
    len[k] = it[lo + k].len;
    pos += packed_len(it[lo + k]);
  }
  auto copy = [&](uint32_t a, uint32_t b) {
    for (uint32_t k = a; k < b; k++) {
      const uint64_t l = len[k], o = off[k];
      memcpy(h + o, it[lo + k].p, l);
      memset(h + o + l, 0, ((l + 7) & ~7ull) - l);
    }
  };
  // MV_PACK_THREADS: host threads packing a large chunk (0: min(8, cores))
  const unsigned hw = std::thread::hardware_concurrency();
  const unsigned max_thr = pack_threads > 0 ? (unsigned)pack_threads : std::min(8u, hw ? hw : 4u);
  const unsigned threads = pos < (8u << 20) ? 1u : std::min<unsigned>(max_thr, m);
  if (threads <= 1) {
    copy(0, m);
  } else {  // item ranges of about equal bytes
    std::vector<std::thread> th;
    uint32_t a = 0;
    for (unsigned t = 1; t <= threads; t++) {
      const uint64_t target = pos * t / threads;
      uint32_t b = a;
      while (b < m && off[b] < target) b++;
      if (t == threads) b = m;
      if (b > a) {
        if (t == threads) copy(a, b);
        else th.emplace_back(copy, a, b);
      }
      a = b;
    }
    for (auto& x : th) x.join();
  }
  memset(h + pos, 0, buf_bytes - pos);
}

mv_status ensure_pass_set(mv_ctx* ctx, Device& dev, int s) {
  Device::PassSet& ps = dev.pset[s];
  if (!ps.stream) {  // a stream of its own: not the host-buffer signature path's copy / compute streams
    if (!dev.qstream[s]) HIPCHK(ctx, hipStreamCreateWithFlags(&dev.qstream[s], hipStreamNonBlocking));
    ps.stream = dev.qstream[s];
  }
  if (!ps.done) HIPCHK(ctx, hipEventCreateWithFlags(&ps.done, hipEventDisableTiming));
  return MV_OK;
}

bool host_pinned(const void* p);
bool pinned_range_holds(const void* p, uint64_t bytes);

// Packs items [lo, hi) into pass set s of dev and enqueues the device pipeline on its stream
// (no wait). The set must be idle. A large chunk whose blocks already lie in page-locked
// caller memory (mv_host_alloc), in order with small gaps, skips the host pack: the DMA engine
// reads the caller's bytes in place (only the offset / length arrays are staged), so the
// host's memory bandwidth is not spent on a second copy.
mv_status enqueue_block_chunk(mv_ctx* ctx, Device& dev, int s, const BlockItem* it, uint64_t lo, uint64_t hi) {
  HIPCHK(ctx, hipSetDevice(dev.id));
  mv_status rc = ensure_pass_set(ctx, dev, s);
  if (rc != MV_OK) return rc;
  Device::PassSet& ps = dev.pset[s];
  const bool trace = ctx->kn.blk_trace != 0;  // diagnostics (MV_BLK_TRACE): host-side times
  auto now = [] { return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
  const double t0 = trace ? now() : 0;
  const uint32_t m = (uint32_t)(hi - lo);
  uint64_t bytes = 0;
  for (uint64_t k = lo; k < hi; k++) bytes += packed_len(it[k]);
  // small chunks (the online path): the ingest kernel reads the pinned staging over PCIe
  // itself (zero-copy) instead of waiting for an H2D copy and the launch behind it
  const uint64_t zc_max = (uint64_t)std::max<int64_t>(0, ctx->kn.blk_zerocopy);  // MV_BLK_ZEROCOPY=<bytes> (0: always copy)
  // in-place DMA of pinned caller bytes (see above)
  const uint8_t* base = it[lo].p;
  uint64_t span = 0;
  bool direct = bytes > zc_max && host_pinned(base);
  for (uint64_t k = lo; k < hi && direct; k++) {
    if (it[k].p < base || (uint64_t)(it[k].p - base) < span) direct = false;  // in order, no overlap
    span = (uint64_t)(it[k].p - base) + it[k].len;
  }
  // any alignment (the ingest kernels read from the aligned word at or below a block's start);
  // gaps between blocks are copied too, so they must stay small
  // ... and [base, base + span) must lie inside ONE page-locked allocation: a pass merges
  // several callers' items, and two callers' buffers may sit close together with unpinned (or
  // unmapped) memory between them
  direct = direct && span && span <= 2 * bytes + 4096 && pinned_range_holds(base, span);
  const size_t buf_bytes = direct ? (span + 16 + 15) & ~(size_t)15 : (bytes + 16 + 15) & ~(size_t)15;
  const size_t o_off = buf_bytes, o_len = o_off + 8 * (size_t)m, total = o_len + 8 * (size_t)m;
  HIPCHK(ctx, ps.h_in.ensure(direct ? 16 * (size_t)m : total));
  uint8_t* h = ps.h_in.as<uint8_t>();
  if (direct) {
    uint64_t* hoff = reinterpret_cast<uint64_t*>(h);
    uint64_t* hlen = hoff + m;
    for (uint32_t k = 0; k < m; k++) {
      hoff[k] = (uint64_t)(it[lo + k].p - base);
      hlen[k] = it[lo + k].len;
    }
  } else {
    pack_items(h, (uint64_t*)(h + o_off), (uint64_t*)(h + o_len), it, lo, hi, buf_bytes, ctx->kn.pack_threads);
  }
  HIPCHK(ctx, ps.bytes.ensure(total));
  HIPCHK(ctx, ps.out2.ensure(65 * (size_t)m + 256));
  HIPCHK(ctx, ps.h_out.ensure(65 * (size_t)m));
  const double t1 = trace ? now() : 0;
  const uint8_t* dbuf = nullptr;
  uint8_t* hout_dev = nullptr;  // zero-copy outputs too: the kernels write the pinned h_out
  if (direct) {
    uint8_t* d = ps.bytes.as<uint8_t>();
    HIPCHK(ctx, hipMemcpyAsync(d, base, span, hipMemcpyHostToDevice, ps.stream));
    HIPCHK(ctx, hipMemsetAsync(d + span, 0, buf_bytes - span, ps.stream));  // the 16 readable bytes past the end
    HIPCHK(ctx, hipMemcpyAsync(d + o_off, h, 16 * (size_t)m, hipMemcpyHostToDevice, ps.stream));
    dbuf = d;
  } else if (total <= zc_max) {
    void* dp = nullptr;
    void* dq = nullptr;
    // outputs only under the comb path: the batch path re-reads the digests many times
    const bool zc_out = m < MV_BATCH_MIN;
    if (hipHostGetDevicePointer(&dp, h, 0) == hipSuccess && dp &&
        (!zc_out || (hipHostGetDevicePointer(&dq, ps.h_out.p, 0) == hipSuccess && dq))) {
      dbuf = static_cast<const uint8_t*>(dp);
      hout_dev = static_cast<uint8_t*>(dq);
    } else {
      (void)hipGetLastError();
    }
  }
  if (!dbuf) {
    HIPCHK(ctx, hipMemcpyAsync(ps.bytes.p, h, total, hipMemcpyHostToDevice, ps.stream));
    dbuf = ps.bytes.as<uint8_t>();
  }
  const double t2 = trace ? now() : 0;
  uint8_t* dout = hout_dev ? hout_dev : ps.out2.as<uint8_t>();
  rc = enqueue_blocks(ctx, dev, dbuf, buf_bytes, (const uint64_t*)(dbuf + o_off), (const uint64_t*)(dbuf + o_len), m,
                      dout + 64 * (size_t)m, dout, dout + 32 * (size_t)m, ps.stream, &ps.scr, &ps.aux);
  if (rc != MV_OK) {
    (void)hipStreamSynchronize(ps.stream);  // what was queued reads the staging
    return rc;
  }
  // from here on an error must drain the stream first: the queued kernels read the staging
  hipError_t e = hout_dev ? hipSuccess : hipMemcpyAsync(ps.h_out.p, dout, 65 * (size_t)m, hipMemcpyDeviceToHost, ps.stream);
  if (e == hipSuccess) e = hipEventRecord(ps.done, ps.stream);
  if (e != hipSuccess) {
    (void)hipStreamSynchronize(ps.stream);
    return set_err(ctx, MV_E_HIP, std::string("block pass: ") + hipGetErrorString(e));
  }
  ps.it = it;
  ps.lo = lo;
  ps.m = m;
  ps.inflight = true;
  if (trace)
    fprintf(stderr, "[blk] set %d, %u blocks%s: pack %.1f, h2d %.1f, kernels %.1f us\n", s, m, direct ? " (in place)" : "",
            t1 - t0, t2 - t1, now() - t2);
  return MV_OK;
}

// Waits for pass set s's chunk and scatters its verdicts and digests to the blocks' owners.
// Needs no context lock (the set is owned by the caller until it is marked idle).
mv_status finish_block_chunk(mv_ctx* ctx, Device& dev, int s) {
  Device::PassSet& ps = dev.pset[s];
  if (!ps.inflight) return MV_OK;
  ps.inflight = false;
  HIPCHK(ctx, hipSetDevice(dev.id));
  // MV_PASS_SPIN=1 (A/B): the pass owner polls its event instead of blocking in the runtime
  const bool spin = ctx->kn.pass_spin != 0;
  hipError_t e;
  if (spin) {
    while ((e = hipEventQuery(ps.done)) == hipErrorNotReady) std::this_thread::yield();
  } else {
    e = hipEventSynchronize(ps.done);
  }
  if (e != hipSuccess) {
    (void)hipStreamSynchronize(ps.stream);
    return set_err(ctx, MV_E_HIP, std::string("block pass: ") + hipGetErrorString(e));
  }
  const BlockItem* it = static_cast<const BlockItem*>(ps.it);
  const uint32_t m = ps.m;
  const uint8_t* ho = ps.h_out.as<uint8_t>();
  for (uint32_t k = 0; k < m; k++) {
    const BlockItem& b = it[ps.lo + k];
    *b.st = ho[64 * (size_t)m + k];
    if (b.md) memcpy(b.md, ho + 32 * (size_t)k, 32);
    if (b.bd) memcpy(b.bd, ho + 32 * ((size_t)m + k), 32);
  }
  return MV_OK;
}

// Items [lo, hi) on dev in chunks over both pass sets (chunk c + 1 packed and enqueued while
// chunk c runs); returns when all are scattered. Caller holds ctx->mu and owns both sets.
mv_status verify_block_items(mv_ctx* ctx, Device& dev, const BlockItem* it, uint64_t lo, uint64_t hi) {
  mv_status rc = MV_OK;
  int s = 0;
  for (uint64_t i = lo; i < hi && rc == MV_OK; s ^= 1) {
    rc = finish_block_chunk(ctx, dev, s);  // the set's chunk before last
    if (rc != MV_OK) break;
    const uint64_t j = chunk_end(ctx, it, i, hi);
    rc = enqueue_block_chunk(ctx, dev, s, it, i, j);
    i = j;
  }
  for (int k = 0; k < 2; k++) {
    const mv_status r2 = finish_block_chunk(ctx, dev, k);
    if (rc == MV_OK) rc = r2;
  }
  poll_flags(ctx, dev);
  return rc;
}

bool committee_ready(mv_ctx* ctx) {
  if (!ctx->has_committee) return false;
  for (auto& dev : ctx->devs)
    if (!dev.committee_loaded) return false;
  return true;
}

// ---- the resident online service (kernels.h k_online) -------------------------------------
// One per device, made on the first eligible request. Page-locked coherent host memory holds
// the control words, the request ring and each slot's bincode in / outputs out (the kernel
// reads and writes them over PCIe, as the launched online path does); device memory holds the
// ticket and each slot's ingest scratch. The kernel runs on its own stream, the engine's only
// one of the highest priority (a queue of its own, so kernels on other streams never wait behind
// it; its 64 workgroups bound its share of the chip), and exits after MV_ONLINE_IDLE_US (default
// 10,000) without a job.
constexpr uint32_t kOnSlots = mvk::ONLINE_SLOTS, kOnMax = mvk::ONLINE_MAX_BLOCKS;
constexpr size_t kOnInCap = mvk::ONLINE_IN_CAP;        // bincode bytes per request
constexpr size_t kOnInStride = mvk::ONLINE_IN_STRIDE;  // off[n] | len[n] | bincode | 16 zero B
constexpr size_t kOnOutStride = mvk::ONLINE_OUT_STRIDE;  // md[64] | bd[64] | status[64]

struct OnlineSvc {
  std::mutex mu;
  bool ready = false, launched = false;
  // set once the service cannot serve (a failed launch, a timed-out request): later requests
  // take the submission queue; read without o.mu by callers waiting for a slot or a verdict
  std::atomic<bool> failed{false};
  bool stuck = false;  // a launch that would not end: its stream and memory are never released
  hipStream_t stream = nullptr;
  hipEvent_t exited = nullptr;
  mvk::OnlineCtl* ctl = nullptr;  // host view (pinned, coherent)
  mvk::OnlineReq* req = nullptr;
  uint8_t* in = nullptr;
  uint8_t* out = nullptr;
  void *ctl_d = nullptr, *req_d = nullptr, *in_d = nullptr, *out_d = nullptr;  // device views
  DevBuf dctl, scr;
  std::unique_ptr<std::atomic<uint64_t>[]> freed;  // slot released by its owner: request + 1
  // Waiting callers (round 5). At most max_spinners callers spin on their done word; the others
  // sleep on a futex word of their slot, which the reaper thread sets and wakes once the done
  // word holds their request (99 callers spinning on a 16-CPU share descheduled one another
  // for milliseconds: p99 81 ms). A caller waiting for its slot to be freed sleeps the same way.
  int max_spinners = 4;
  std::atomic<int> spinners{0}, sleepers{0};
  std::unique_ptr<std::atomic<uint32_t>[]> dwake;  // per slot: set by the reaper (futex word)
  std::unique_ptr<std::atomic<uint64_t>[]> sleep_q;  // per slot: request + 1 its sleeper waits for, 0: none
  std::unique_ptr<std::atomic<uint32_t>[]> fseq, fwait;  // per slot: frees so far (futex word), sleepers on it
  std::thread reaper;
  std::mutex rmu;
  std::condition_variable rcv;
  bool rstop = false;
  uint64_t next_q = 0;
  uint32_t grid = 0, launch_no = 0;
  std::atomic<uint64_t> requests{0}, launches{0};
  uint64_t idle_us = 10000;
  // MV_ONLINE_TRACE: per-stage sums (us) -- host publish to done seen, and on the kernel's
  // clock seen -> ready -> first claim -> last job done -- printed at release
  bool trace = false, debug = false;  // MV_ONLINE_TRACE, MV_ONLINE_DEBUG
  double ticks_per_us = 100.0;
  std::mutex tr_mu;
  double tr_sum[14] = {};
  uint64_t tr_n = 0;
};

int64_t steady_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

// Whether a request of n blocks, `bytes` of 8-aligned bincode, takes the online service: the
// calls enqueue_blocks would run as one k_verify_comb16 launch (short blocks, the ingest and
// hash folded in), small enough for one ring slot.
// Long blocks (config-4 shape, ~9.5 KB) take the service too: a request is then one job whose
// A wave hashes the whole pre-image (the R decode runs beside it), against the queue's split
// launch pair: 16 one-block config-4-shape callers 80.8-81.0 k blocks/s, p50 197-198 us, against
// 69.4-70.6 k / 223-225 us (profiles/r04/c5_online_long_r04s.txt). MV_ONLINE_LONG=0: short
// blocks only (< MV_COMB_SPLIT_BYTES on average, as the queue's one-launch case). A block past
// the wave-parallel ingest's LDS window (ingest_dev.h IG_WIN) goes through the queue.
bool online_eligible(mv_ctx* ctx, uint32_t n, uint64_t bytes, uint64_t longest) {
  const mvk::Knobs& kn = ctx->kn;
  if ((ctx->flags & (MV_FLAG_NO_ONLINE | MV_FLAG_NO_COMB | MV_FLAG_HOST_PARSE)) || !kn.online) return false;
  if (n == 0 || n > kOnMax || bytes > kOnInCap) return false;
  if (longest + 32 > mvk::INGEST_WINDOW_BYTES) return false;
  const uint64_t split_bytes = (uint64_t)std::max<int64_t>(0, kn.comb_split_bytes);
  const uint64_t buf_bytes = (bytes + 16 + 15) & ~15ull;
  if (!kn.online_long && split_bytes && buf_bytes >= split_bytes * (uint64_t)n) return false;
  if (!kn.hash_in_comb || !kn.ingest_in_comb) return false;
  return mvk::comb_short_chain(kn, n);
}

void futex_wait_for(std::atomic<uint32_t>& w, uint32_t v, int64_t ns) {
  static_assert(sizeof(std::atomic<uint32_t>) == 4, "futex word");
  timespec ts{(time_t)(ns / 1000000000), (long)(ns % 1000000000)};
  (void)syscall(SYS_futex, reinterpret_cast<uint32_t*>(&w), FUTEX_WAIT_PRIVATE, v, &ts, nullptr, 0);
}
void futex_wake_all(std::atomic<uint32_t>& w) {
  (void)syscall(SYS_futex, reinterpret_cast<uint32_t*>(&w), FUTEX_WAKE_PRIVATE, INT_MAX, nullptr, nullptr, 0);
}

// CPUs this process may use: its affinity mask, capped by a cgroup-v2 CPU quota.
int host_cpu_share() {
  cpu_set_t set;
  int n = sched_getaffinity(0, sizeof(set), &set) == 0 ? CPU_COUNT(&set) : (int)std::thread::hardware_concurrency();
  if (FILE* f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
    char quota[32] = {0};
    long period = 0;
    if (fscanf(f, "%31s %ld", quota, &period) == 2 && strcmp(quota, "max") != 0 && period > 0) {
      const long q = atol(quota);
      if (q > 0) n = std::min<int>(n, (int)std::max<long>(1, q / period));
    }
    fclose(f);
  }
  return std::max(1, n);
}

// Wakes the sleeping callers whose done word is set (one thread per service, started with it;
// it polls only while callers sleep and otherwise waits on rcv).
void online_reaper(OnlineSvc* op) {
  OnlineSvc& o = *op;
  std::unique_lock<std::mutex> lk(o.rmu);
  while (!o.rstop) {
    if (o.sleepers.load(std::memory_order_acquire) == 0) {
      o.rcv.wait_for(lk, std::chrono::milliseconds(20));
      continue;
    }
    lk.unlock();
    for (int it = 0; it < 4096 && o.sleepers.load(std::memory_order_relaxed) > 0; it++) {
      for (uint32_t k = 0; k < kOnSlots; k++) {
        uint64_t w = o.sleep_q[k].load(std::memory_order_acquire);
        if (w && __atomic_load_n(&o.ctl->done[k], __ATOMIC_ACQUIRE) == w &&
            o.sleep_q[k].compare_exchange_strong(w, 0, std::memory_order_acq_rel)) {
          o.dwake[k].store(1, std::memory_order_release);
          futex_wake_all(o.dwake[k]);
        }
      }
      __builtin_ia32_pause();
    }
    lk.lock();
  }
}

// Allocations and the stream (o.mu held).
mv_status online_init(mv_ctx* ctx, Device& dev, OnlineSvc& o) {
  if (o.ready) return MV_OK;
  HIPCHK(ctx, hipSetDevice(dev.id));
  const unsigned fl = hipHostMallocMapped | hipHostMallocCoherent | hipHostMallocPortable;
  auto host = [&](void** h, void** d, size_t bytes) -> hipError_t {
    hipError_t e = hipHostMalloc(h, bytes, fl);
    if (e != hipSuccess) return e;
    memset(*h, 0, bytes);
    return hipHostGetDevicePointer(d, *h, 0);
  };
  HIPCHK(ctx, host((void**)&o.ctl, &o.ctl_d, sizeof(mvk::OnlineCtl)));
  HIPCHK(ctx, host((void**)&o.req, &o.req_d, sizeof(mvk::OnlineReq) * kOnSlots));
  HIPCHK(ctx, host((void**)&o.in, &o.in_d, kOnInStride * kOnSlots));
  HIPCHK(ctx, host((void**)&o.out, &o.out_d, kOnOutStride * kOnSlots));
  HIPCHK(ctx, o.dctl.ensure(sizeof(mvk::OnlineDev)));
  HIPCHK(ctx, hipMemset(o.dctl.p, 0, sizeof(mvk::OnlineDev)));
  HIPCHK(ctx, o.scr.ensure(mvk::ONLINE_SCR_STRIDE * kOnSlots));
  o.freed.reset(new std::atomic<uint64_t>[kOnSlots]);
  o.dwake.reset(new std::atomic<uint32_t>[kOnSlots]);
  o.sleep_q.reset(new std::atomic<uint64_t>[kOnSlots]);
  o.fseq.reset(new std::atomic<uint32_t>[kOnSlots]);
  o.fwait.reset(new std::atomic<uint32_t>[kOnSlots]);
  for (uint32_t k = 0; k < kOnSlots; k++) {
    o.freed[k].store(0);
    o.dwake[k].store(0);
    o.sleep_q[k].store(0);
    o.fseq[k].store(0);
    o.fwait[k].store(0);
  }
  o.max_spinners = ctx->kn.online_spinners > 0 ? (int)ctx->kn.online_spinners
                                               : std::max(1, host_cpu_share() / 4);
  if (!o.reaper.joinable()) {
    o.rstop = false;
    o.reaper = std::thread(online_reaper, &o);
  }
  // The service's stream needs a hardware queue of its own: a kernel queued behind the resident
  // one on a shared queue would wait for it. A stream of the highest priority (the runtime keeps
  // a queue per priority level, and the engine's other streams are all of the default
  // priority). Round 4 used a CU-masked stream: tearing one down left a later hipStreamDestroy
  // of an unrelated stream waiting forever on a runtime lock in about 1 of 10 processes
  // (the driver's round-4 smoke); that form was removed in round 6.
  // MV_ONLINE_PRIO = 0: an ordinary stream (shares a queue; A/B only).
  if (ctx->kn.online_prio) {
    int least = 0, greatest = 0;
    HIPCHK(ctx, hipDeviceGetStreamPriorityRange(&least, &greatest));
    HIPCHK(ctx, hipStreamCreateWithPriority(&o.stream, hipStreamNonBlocking, greatest));
  } else {
    HIPCHK(ctx, hipStreamCreateWithFlags(&o.stream, hipStreamNonBlocking));
  }
  HIPCHK(ctx, hipEventCreateWithFlags(&o.exited, hipEventDisableTiming));
  o.trace = ctx->kn.online_trace != 0;
  o.debug = ctx->kn.online_debug != 0;
  {
    int khz = 0;
    if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev.id) == hipSuccess && khz > 0)
      o.ticks_per_us = khz / 1000.0;
    else
      (void)hipGetLastError();
  }
  const int64_t ge = ctx->kn.online_wgs;  // resident workgroups (4-block jobs in flight; 0: 64)
  o.grid = (uint32_t)(ge > 0 ? std::max<int64_t>(2, ge) : 64);  // >= 2: the poller + workers
  o.grid = std::min<uint32_t>(o.grid, mvk::ONLINE_MAX_WGS);
  o.ready = true;
  return MV_OK;
}

// Launches the kernel unless one is live (o.mu held).
mv_status online_ensure_running(mv_ctx* ctx, Device& dev, OnlineSvc& o) {
  if (o.launched) {
    // the poller's liveness word (comb.hip k_online): the launch number while it runs,
    // | ONLINE_WG_LEFT once it has left -- no runtime query on the request path. An older
    // value means the launch has not started yet: it will see the request.
    const uint32_t w = __atomic_load_n(&o.ctl->wg[0], __ATOMIC_ACQUIRE);
    if (w != (o.launch_no | mvk::ONLINE_WG_LEFT)) return MV_OK;
  }
  if (ctx->kn.online_inject) {  // fault injection (tests): the launch fails
    (void)hipGetLastError();
    return set_err(ctx, MV_E_HIP, "online service: injected launch failure (MV_ONLINE_INJECT)");
  }
  if (o.launched) {
    const hipError_t q = hipEventQuery(o.exited);
    if (q == hipErrorNotReady) {
      (void)hipGetLastError();
      return MV_OK;  // still running
    }
    if (q != hipSuccess) {
      o.failed = true;
      return set_err(ctx, MV_E_HIP, std::string("online service: ") + hipGetErrorString(q));
    }
  }
  const uint64_t idle_us = (uint64_t)std::max<int64_t>(0, ctx->kn.online_idle_us);
  o.idle_us = idle_us;
  __atomic_store_n(&o.ctl->stop, 0ull, __ATOMIC_RELEASE);
  HIPCHK(ctx, hipSetDevice(dev.id));
  // the kernel's wall clock (s_memrealtime) in kHz; a launch lives at most 60 s (callers relaunch)
  int khz = 0;
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev.id) != hipSuccess || khz <= 0) {
    (void)hipGetLastError();
    khz = 100000;
  }
  const uint64_t per_us = (uint64_t)khz / 1000 ? (uint64_t)khz / 1000 : 1;
  mvk::OnlineArgs a{};
  a.ctl = (mvk::OnlineCtl*)o.ctl_d;
  a.reqs = (const mvk::OnlineReq*)o.req_d;
  a.dev = o.dctl.as<mvk::OnlineDev>();
  a.in_host = static_cast<const uint8_t*>(o.in_d);
  a.out_host = static_cast<uint8_t*>(o.out_d);
  a.scr = o.scr.as<uint8_t>();
  a.combB = dev.combB.p;
  a.combA = dev.combA.p;
  a.key_ok = dev.keyok.as<uint8_t>();
  a.pk = dev.committee_pk.as<uint8_t>();
  a.stakes = dev.stakes.as<uint64_t>();
  const mvh::Committee& com = ctx->committee;  // fixed while the launch lives (mv_set_committee stops it)
  a.epoch = com.epoch;
  a.quorum_thr = com.quorum_threshold;
  a.n_auth = (uint32_t)com.size();
  a.launch = ++o.launch_no;
  a.idle_ticks = idle_us * per_us;
  a.max_ticks = 60000000ull * per_us;
  HIPCHK(ctx, mvk::launch_online(a, o.grid, o.stream));
  if (o.debug)
    fprintf(stderr, "[online] launch %u: grid %u, idle %llu us, wall clock %d kHz\n", a.launch, o.grid,
            (unsigned long long)idle_us, khz);
  HIPCHK(ctx, hipEventRecord(o.exited, o.stream));
  o.launched = true;
  o.launches++;
  return MV_OK;
}

// Polls ev until it completes or limit_ms pass (no blocking runtime wait, which cannot be
// bounded); true once complete.
bool event_done_within(hipEvent_t ev, int64_t limit_ms) {
  const int64_t t0 = steady_ns();
  for (;;) {
    const hipError_t q = hipEventQuery(ev);
    if (q == hipSuccess) return true;
    (void)hipGetLastError();
    if (q != hipErrorNotReady) return true;  // an error: nothing more will complete on it
    if (steady_ns() - t0 > limit_ms * 1000000) return false;
    std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
}

// The service's state words, for a launch that does not end in time (stderr).
void online_dump(const OnlineSvc& o, const char* why) {
  const mvk::OnlineCtl* c = o.ctl;
  uint32_t running = 0, left = 0, other = 0;
  std::string stuck;
  for (uint32_t g = 0; g < o.grid && g < mvk::ONLINE_MAX_WGS; g++) {
    const uint32_t w = __atomic_load_n(&c->wg[g], __ATOMIC_ACQUIRE);
    if (w == o.launch_no) {
      running++;
      if (stuck.size() < 96) stuck += " " + std::to_string(g);
    } else if (w == (o.launch_no | mvk::ONLINE_WG_LEFT)) {
      left++;
    } else {
      other++;
    }
  }
  fprintf(stderr,
          "[online] %s: launch %u grid %u: %u workgroups running (%s), %u left, %u not started; stop %llu tail %llu "
          "next_q %llu; poller exit: why %llu ready %llu jobs_head %llu jobs_tail %llu\n",
          why, o.launch_no, o.grid, running, stuck.empty() ? "-" : stuck.c_str() + 1, left, other,
          (unsigned long long)c->stop, (unsigned long long)c->tail, (unsigned long long)o.next_q,
          (unsigned long long)c->exit_why, (unsigned long long)c->exit_ready, (unsigned long long)c->exit_head,
          (unsigned long long)c->exit_tail);
}

// Stops the kernel once it is idle and waits for it, bounded (o.mu held). The launch's own
// limits end every wave within max_ticks + idle (60 s + MV_ONLINE_IDLE_US); a launch still
// running well past that is reported (online_dump) and the service is left stuck: its memory is
// then never freed (the kernel may still touch it). Returns false in that case.
bool online_stop(OnlineSvc& o) {
  if (!o.ready || !o.launched) return true;
  __atomic_store_n(&o.ctl->stop, 1ull, __ATOMIC_RELEASE);
  bool done = event_done_within(o.exited, 2000);
  if (!done) {
    online_dump(o, "stop: no exit after 2 s");
    done = event_done_within(o.exited, 70000);
    if (!done) online_dump(o, "stop: no exit after 72 s, service abandoned");
  }
  if (!done) {
    o.failed = o.stuck = true;
    return false;
  }
  __atomic_store_n(&o.ctl->stop, 0ull, __ATOMIC_RELEASE);
  o.launched = false;
  return true;
}

void online_release(OnlineSvc& o) {
  if (o.reaper.joinable()) {
    {
      std::lock_guard<std::mutex> lk(o.rmu);
      o.rstop = true;
    }
    o.rcv.notify_all();
    o.reaper.join();
  }
  if (!online_stop(o)) return;  // stuck: leave its stream and memory alone
  if (o.trace && o.tr_n) {
    const double n = (double)o.tr_n;
    fprintf(stderr,
            "[online] %llu requests, mean us: host publish->done seen %.1f | kernel: seen->ready %.1f, "
            "ready->claim %.1f, claim->done %.1f, seen->done %.1f | job 0 from its claim: barrier 0 %.1f, "
            "B rows %.1f, S %.1f, R decoded %.1f, barrier 1 %.1f, verdict %.1f, fenced %.1f, digests %.1f, "
            "k %.1f\n",
            (unsigned long long)o.tr_n, o.tr_sum[0] / n, o.tr_sum[1] / n, o.tr_sum[2] / n, o.tr_sum[3] / n,
            o.tr_sum[4] / n, o.tr_sum[5] / n, o.tr_sum[6] / n, o.tr_sum[7] / n, o.tr_sum[8] / n, o.tr_sum[9] / n,
            o.tr_sum[10] / n, o.tr_sum[11] / n, o.tr_sum[12] / n, o.tr_sum[13] / n);
  }
  if (o.stream) (void)hipStreamDestroy(o.stream);
  if (o.exited) (void)hipEventDestroy(o.exited);
  for (void* h : {(void*)o.ctl, (void*)o.req, (void*)o.in, (void*)o.out})
    if (h) (void)hipHostFree(h);
  o.dctl.release();
  o.scr.release();
  o.ready = false;
}

// One request through the service: reserve a ring slot, pack the blocks into its page-locked
// input, publish the descriptor, then poll the slot's done word (the caller's thread spins:
// no launch, no event, no wake-up). ctx->com_mu is held shared by the caller.
mv_status online_verify(mv_ctx* ctx, Device& dev, const uint8_t* buf, const uint64_t* off, const uint64_t* len,
                        uint32_t n, uint8_t* status, uint8_t* md, uint8_t* bd) {
  OnlineSvc& o = *dev.online;
  uint64_t q;
  {
    std::lock_guard<std::mutex> lk(o.mu);
    if (o.failed) return set_err(ctx, MV_E_HIP, "online service failed earlier");
    mv_status rc = online_init(ctx, dev, o);
    if (rc != MV_OK) {
      o.failed = true;
      return rc;
    }
    q = o.next_q++;
    __atomic_store_n(&o.ctl->tail, o.next_q, __ATOMIC_RELEASE);
    rc = online_ensure_running(ctx, dev, o);
    if (rc != MV_OK) {
      // request q is never published, so the poller would stop at it: the service is done
      // (every later reservation sees `failed`, every waiting caller leaves its loop)
      o.failed = true;
      return rc;
    }
  }
  o.requests++;
  const uint32_t slot = (uint32_t)(q % kOnSlots);
  if (q >= kOnSlots) {  // the slot's previous request must have been read out by its owner
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t spins = 0; o.freed[slot].load(std::memory_order_acquire) != q - kOnSlots + 1; spins++) {
      // the owner of request q - 64 failed (its service failed with it) or never returns
      if (o.failed.load(std::memory_order_relaxed) || std::chrono::steady_clock::now() - t0 > std::chrono::seconds(20)) {
        o.failed = true;
        return set_err(ctx, MV_E_HIP, "online service failed: ring slot never released");
      }
      if (spins < 256) {
        __builtin_ia32_pause();
        continue;
      }
      // sleep until the owner frees the slot (it wakes fseq's sleepers), 1 ms at most
      const uint32_t seen = o.fseq[slot].load(std::memory_order_acquire);
      o.fwait[slot].fetch_add(1, std::memory_order_acq_rel);
      if (o.freed[slot].load(std::memory_order_acquire) != q - kOnSlots + 1) futex_wait_for(o.fseq[slot], seen, 1000000);
      o.fwait[slot].fetch_sub(1, std::memory_order_acq_rel);
    }
  }
  // the slot's input: off[n] | len[n] | bincode (8-aligned blocks) | 16 zero bytes; the poller
  // copies it to the slot's HBM scratch, which every device pointer below refers to
  uint8_t* in = o.in + kOnInStride * slot;
  uint64_t* hoff = reinterpret_cast<uint64_t*>(in);
  uint64_t* hlen = hoff + n;
  uint8_t* bytes = in + 16 * (size_t)n;
  uint64_t pos = 0;
  for (uint32_t k = 0; k < n; k++) {
    const uint64_t l = len[k];
    hoff[k] = pos;
    hlen[k] = l;
    memcpy(bytes + pos, buf + off[k], l);
    const uint64_t pl = (l + 7) & ~7ull;
    memset(bytes + pos + l, 0, pl - l);
    pos += pl;
  }
  memset(bytes + pos, 0, 16);  // 16 readable zero bytes past the last block
  const uint32_t copy_bytes = (uint32_t)((16 * (size_t)n + pos + 16 + 15) & ~(size_t)15);
  uint8_t* out = o.out + kOnOutStride * slot;
  mvk::OnlineReq& r = o.req[slot];
  r.n = n;
  r.copy_bytes = copy_bytes;
  const int64_t t_pub = o.trace ? steady_ns() : 0;
  __atomic_store_n(&r.seq, q + 1, __ATOMIC_RELEASE);  // the descriptor and the bytes above first
  // wait for the slot's done word, spinning (at most max_spinners callers at once) or asleep
  // until the reaper wakes it; every ~100 us (asleep: 1 ms) check that a kernel is still live
  // (one that exited idle just before this request was published is relaunched)
  auto t_last = std::chrono::steady_clock::now();
  const auto t_start = t_last;
  mv_status rc = MV_OK;
  auto is_done = [&] { return __atomic_load_n(&o.ctl->done[slot], __ATOMIC_ACQUIRE) == q + 1; };
  auto check = [&](std::chrono::steady_clock::time_point now) -> bool {  // false: give up (rc set)
    if (o.debug && now - t_start > std::chrono::milliseconds(500) &&
        (now - t_start) % std::chrono::milliseconds(500) < std::chrono::milliseconds(2)) {
      const uint64_t* tr = o.ctl->trace[slot];
      fprintf(stderr, "[online] q %llu slot %u waiting %.1f ms: done %llu seq %llu tail %llu trace %llu %llu %llu %llu\n",
              (unsigned long long)q, slot,
              std::chrono::duration<double, std::milli>(now - t_start).count(),
              (unsigned long long)__atomic_load_n(&o.ctl->done[slot], __ATOMIC_ACQUIRE),
              (unsigned long long)o.req[slot].seq, (unsigned long long)o.ctl->tail, (unsigned long long)tr[0],
              (unsigned long long)tr[1], (unsigned long long)tr[2], (unsigned long long)tr[3]);
    }
    std::lock_guard<std::mutex> lk(o.mu);
    if (o.failed) {
      rc = set_err(ctx, MV_E_HIP, "online service failed");
      return false;
    }
    rc = online_ensure_running(ctx, dev, o);
    if (rc == MV_OK && o.launched && now - t_start > std::chrono::microseconds(std::max<uint64_t>(o.idle_us, 1000))) {
      // waiting longer than the idle limit: a launch that faulted or was aborted never marks its
      // liveness word LEFT, so ask the runtime about its end as well (fail fast, not after 20 s)
      const hipError_t q = hipEventQuery(o.exited);
      if (q == hipErrorNotReady)
        (void)hipGetLastError();
      else if (q != hipSuccess)
        rc = set_err(ctx, MV_E_HIP, std::string("online service: ") + hipGetErrorString(q));
    }
    if (rc == MV_OK && now - t_start > std::chrono::seconds(20))
      rc = set_err(ctx, MV_E_HIP, "online service: request timed out");
    if (rc != MV_OK) {
      o.failed = true;  // the slot may still be written: never reuse the service
      return false;
    }
    return true;
  };
  if (o.spinners.fetch_add(1, std::memory_order_acq_rel) < o.max_spinners) {
    for (uint32_t spins = 0; !is_done();) {
      if (++spins < 64) {
        __builtin_ia32_pause();
        continue;
      }
      spins = 0;
      std::this_thread::yield();
      const auto now = std::chrono::steady_clock::now();
      if (now - t_last < std::chrono::microseconds(100)) continue;
      t_last = now;
      if (!check(now)) break;
    }
    o.spinners.fetch_sub(1, std::memory_order_acq_rel);
  } else {
    o.spinners.fetch_sub(1, std::memory_order_acq_rel);
    o.dwake[slot].store(0, std::memory_order_relaxed);
    o.sleep_q[slot].store(q + 1, std::memory_order_release);
    if (o.sleepers.fetch_add(1, std::memory_order_acq_rel) == 0) {
      std::lock_guard<std::mutex> lk(o.rmu);
      o.rcv.notify_one();
    }
    while (!is_done()) {
      futex_wait_for(o.dwake[slot], 0, 1000000);
      if (is_done()) break;
      const auto now = std::chrono::steady_clock::now();
      if (now - t_last < std::chrono::microseconds(900)) continue;
      t_last = now;
      if (!check(now)) break;
    }
    uint64_t w = q + 1;
    o.sleep_q[slot].compare_exchange_strong(w, 0, std::memory_order_acq_rel);
    o.sleepers.fetch_sub(1, std::memory_order_acq_rel);
  }
  if (rc != MV_OK) return rc;
  if (o.trace) {
    const double host_us = (steady_ns() - t_pub) / 1e3;
    const uint64_t* tr = o.ctl->trace[slot];
    const double k = 1.0 / o.ticks_per_us;
    std::lock_guard<std::mutex> lk(o.tr_mu);
    o.tr_sum[0] += host_us;
    o.tr_sum[1] += (double)(int64_t)(tr[1] - tr[0]) * k;
    o.tr_sum[2] += (double)(int64_t)(tr[2] - tr[1]) * k;
    o.tr_sum[3] += (double)(int64_t)(tr[3] - tr[2]) * k;
    o.tr_sum[4] += (double)(int64_t)(tr[3] - tr[0]) * k;
    for (int i = 0; i < 9; i++) o.tr_sum[5 + i] += (double)(int64_t)(tr[4 + i] - tr[2]) * k;
    o.tr_n++;
  }
  const uint8_t* ho = out;
  for (uint32_t k = 0; k < n; k++) {
    status[k] = ho[64 * kOnMax + k];
    if (md) memcpy(md + 32 * (size_t)k, ho + 32 * (size_t)k, 32);
    if (bd) memcpy(bd + 32 * (size_t)k, ho + 32 * ((size_t)kOnMax + k), 32);
  }
  o.freed[slot].store(q + 1, std::memory_order_release);
  o.fseq[slot].fetch_add(1, std::memory_order_acq_rel);
  if (o.fwait[slot].load(std::memory_order_acquire)) futex_wake_all(o.fseq[slot]);
  return MV_OK;
}

// One pass of the submission queue over the requests the combining caller took. set >= 0:
// the pass fits one chunk per device and runs on that pass set: it is packed and enqueued
// under ctx->mu, `enqueued()` is called, and the caller waits for the device without the
// lock (the next pass can be packed meanwhile). set < 0: a large pass that owns both sets
// and streams its chunks (`enqueued()` at the end). Every request gets rc (and err).
template <class Enqueued>
void run_block_requests(mv_ctx* ctx, std::deque<mv_ctx::BlockReq*>& reqs, int set, Enqueued enqueued) {
  bool signalled = false;
  auto signal = [&] {
    if (!signalled) {
      signalled = true;
      enqueued();
    }
  };
  std::string err;
  mv_status rc = MV_OK;
  std::vector<BlockItem> items;
  std::vector<std::pair<size_t, std::pair<uint64_t, uint64_t>>> shards;  // device, [lo, hi)
  try {
    size_t total = 0;
    for (auto* r : reqs) total += r->n;
    items.reserve(total);
    for (auto* r : reqs)
      for (uint32_t k = 0; k < r->n; k++)
        items.push_back(BlockItem{r->buf + r->off[k], r->len[k], r->status + k,
                                  r->md ? r->md + 32 * (size_t)k : nullptr, r->bd ? r->bd + 32 * (size_t)k : nullptr});
    std::lock_guard<std::mutex> lk(ctx->mu);
    ctx->q_passes++;
    t_err = &err;
    const size_t nd = ctx->devs.size();
    std::vector<uint64_t> cut;
    if (nd == 1 || items.size() < 2 * nd) {
      cut = {0, (uint64_t)items.size()};
    } else {
      std::vector<uint64_t> w(items.size());
      for (size_t k = 0; k < items.size(); k++) w[k] = items[k].len + 64;  // bytes, plus a per-block constant
      cut = balanced_cuts(w.data(), w.size(), (uint32_t)nd);
    }
    // the committee is checked again under the lock: a failed mv_set_committee may have
    // unpublished it after the request was queued
    if (!committee_ready(ctx)) {
      rc = set_err(ctx, MV_E_NO_COMMITTEE, "mv_set_committee first");
    } else if (set >= 0) {
      shards.reserve(cut.size());  // push_back below must not throw once a chunk is in flight
      for (size_t d = 0; d + 1 < cut.size() && rc == MV_OK; d++) {
        if (cut[d] == cut[d + 1]) continue;
        rc = enqueue_block_chunk(ctx, ctx->devs[d], set, items.data(), cut[d], cut[d + 1]);
        if (rc == MV_OK) shards.push_back({d, {cut[d], cut[d + 1]}});
      }
    } else if (cut.size() == 2) {
      rc = verify_block_items(ctx, ctx->devs[0], items.data(), 0, items.size());
    } else {
      rc = for_each_cut(ctx, cut, [&](Device& dev, uint64_t lo, uint64_t hi) -> mv_status {
        return verify_block_items(ctx, dev, items.data(), lo, hi);
      });
      if (rc != MV_OK) err = ctx->err;
    }
    t_err = nullptr;
  } catch (...) {  // std::bad_alloc from the item list or the shard plan
    t_err = nullptr;
    rc = MV_E_ALLOC;
    err = "mv_verify_blocks: host allocation failed";
  }
  signal();
  // set >= 0: wait for this pass's chunks (outside the context lock) and scatter the verdicts
  for (auto& sh : shards) {
    t_err = &err;
    const mv_status r2 = finish_block_chunk(ctx, ctx->devs[sh.first], set);
    t_err = nullptr;
    if (rc == MV_OK) rc = r2;
  }
  if (set >= 0 && !shards.empty()) {
    std::lock_guard<std::mutex> lk(ctx->mu);
    for (auto& sh : shards) poll_flags(ctx, ctx->devs[sh.first]);
  }
  for (auto* r : reqs) {
    r->rc = rc;
    if (rc != MV_OK) r->err = err;
  }
}

// True if p is page-locked host memory the DMA engines can read directly (mv_host_alloc,
// hipHostMalloc, hipHostRegister, torch pin_memory).
bool host_pinned(const void* p) {
  if (!p) return false;
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();  // pageable memory: the query fails; do not leave the error set
    return false;
  }
  return a.type == hipMemoryTypeHost;
}

// True if [p, p + bytes) lies inside the one page-locked host allocation that holds p (the
// allocation's address range from the runtime). False when the runtime cannot say.
bool pinned_range_holds(const void* p, uint64_t bytes) {
  if (!host_pinned(p)) return false;
  void* start = nullptr;
  size_t size = 0;
  hipDeviceptr_t q = const_cast<void*>(p);
  if (hipPointerGetAttribute(&start, HIP_POINTER_ATTRIBUTE_RANGE_START_ADDR, q) != hipSuccess ||
      hipPointerGetAttribute(&size, HIP_POINTER_ATTRIBUTE_RANGE_SIZE, q) != hipSuccess || !start || !size) {
    (void)hipGetLastError();
    return false;
  }
  const uintptr_t a = reinterpret_cast<uintptr_t>(start), b = reinterpret_cast<uintptr_t>(p);
  return b >= a && b - a <= size && bytes <= size - (b - a);
}

// mv_ed25519_verify's batch path over [lo, hi) of pinned caller arrays, in a few large
// batches (two by default) on two compute streams. The DMA engines copy a batch's inputs
// chunk by chunk on a copy stream, and k_bv_prep of chunk c starts as soon as chunk c has
// landed, so the PCIe copy overlaps the preparation; batch t + 1's copy and preparation run
// beside batch t's sort, buckets and tail (two input buffers, reuse ordered by events).
// Enqueue only (ctx->mu held): the statuses land in dev.sig_stage[slot], complete once both of
// dev.sig_done[slot] have; the caller waits for them without the lock (mv_ed25519_verify).
mv_status verify_host_streamed(mv_ctx* ctx, Device& dev, const uint8_t* msg, const uint8_t* sig, const uint8_t* pk,
                               const uint32_t* key_idx, uint64_t lo, uint64_t hi, int slot) {
  const int chunk_log2 = (int)std::min<int64_t>(24, std::max<int64_t>(8, ctx->kn.stream_chunk_log2));  // MV_STREAM_CHUNK_LOG2
  const uint64_t m = hi - lo;
  // Batch sizes: shares of the call (MV_STREAM_FRACS, separated by ',' or '/'; default 0.7,0.3). The
  // last batch's prep, sort, buckets and tail follow the last copy, so the shares decrease;
  // every batch is whole 1,024s, >= MV_BATCH_MIN and <= max_batch (more batches when needed).
  // (A streaming MSM -- one batch whose chunks are sorted and bucketed during the copy window --
  // measured slower, 181-198 against 208 M/s, and was removed in round 6: DESIGN.md 13.)
  const std::vector<double> fracs(ctx->kn.stream_fracs, ctx->kn.stream_fracs + ctx->kn.n_stream_fracs);
  std::vector<uint32_t> sizes;
  {
    double tot = 0.0;
    for (double f : fracs) tot += f;
    uint64_t done = 0;
    for (size_t k = 0; k < fracs.size() && done < m; k++) {
      uint64_t want = k + 1 == fracs.size() ? m - done : (((uint64_t)(m * fracs[k] / tot)) + 1023) & ~1023ull;
      if (want < MV_BATCH_MIN) want = MV_BATCH_MIN;
      if (want > m - done) want = m - done;
      if (m - done - want > 0 && m - done - want < MV_BATCH_MIN) want = m - done;  // no runt batch
      if (want > ctx->max_batch) want = ctx->max_batch;
      done += want;
      sizes.push_back((uint32_t)want);
    }
    while (done < m) {  // larger than the shares allow (max_batch): whole max_batch batches
      const uint64_t want = std::min<uint64_t>(m - done, ctx->max_batch);
      sizes.push_back((uint32_t)want);
      done += want;
    }
  }
  uint32_t cap = 0;
  for (uint32_t z : sizes) cap = std::max(cap, z);
  uint32_t chunk = 1u << chunk_log2;
  while ((cap + chunk - 1) / chunk > (uint32_t)Device::kMaxChunks / 2) chunk <<= 1;
  // chunk schedule of a batch of k: the first batch starts with small chunks (2^14, 2^15, ...
  // signatures), so the chip starts preparing after ~40 us of copying instead of a whole chunk's
  auto schedule = [&](int first, uint32_t k) {
    std::vector<uint32_t> cut;
    uint32_t o = 0, c = first ? std::min<uint32_t>(chunk, 1u << 14) : chunk;
    while (o < k) {
      cut.push_back(o);
      o += c;
      if (c < chunk) c *= 2;
    }
    cut.push_back(k);
    return cut;
  };
  const size_t kb = pk ? 32 : 4;  // pk rows or committee key indices
  for (int b = 0; b < 2; b++)
    if (!dev.pstream[b]) HIPCHK(ctx, hipStreamCreateWithFlags(&dev.pstream[b], hipStreamNonBlocking));
  for (int b = 0; b < Device::kPinBufs; b++) {
    if (!dev.pin_free[b]) HIPCHK(ctx, hipEventCreateWithFlags(&dev.pin_free[b], hipEventDisableTiming));
    for (int c = 0; c < Device::kMaxChunks; c++)
      if (!dev.chunk_ev[b][c]) HIPCHK(ctx, hipEventCreateWithFlags(&dev.chunk_ev[b][c], hipEventDisableTiming));
    // (a buffer grown while another call's batch still reads it is retired behind pin_free[b])
    HIPCHK(ctx, dev.pin_msg[b].ensure(32 * (size_t)cap, dev.pin_free[b]));
    HIPCHK(ctx, dev.pin_sig[b].ensure(64 * (size_t)cap, dev.pin_free[b]));
    HIPCHK(ctx, dev.pin_pk[b].ensure(kb * cap, dev.pin_free[b]));
    HIPCHK(ctx, dev.pin_st[b].ensure(cap, dev.pin_free[b]));
  }
  for (int k = 0; k < 2; k++)
    if (!dev.sig_done[slot][k]) HIPCHK(ctx, hipEventCreateWithFlags(&dev.sig_done[slot][k], hipEventDisableTiming));
  HIPCHK(ctx, dev.sig_stage[slot].ensure(m));
  uint8_t* hst = dev.sig_stage[slot].as<uint8_t>();
  bool used[2] = {false, false};
  // copies on the device stream (host-buffer signature calls are serialised by ctx->mu, and the
  // block passes have streams of their own); batch t computes on pstream[t & 1]. mv_create makes
  // these three streams first, so they sit on three distinct hardware queues (GPU_MAX_HW_QUEUES
  // = 4; later streams share queues round-robin, and a copy queued behind another stream's
  // kernels would serialise the pipeline)
  hipStream_t xs = dev.stream;
  uint64_t i = lo;
  for (size_t t = 0; t < sizes.size(); i += sizes[t], t++) {
    // input buffers and compute streams rotate across calls too, so a second caller's first batch
    // copies into a buffer the first caller's batches are not using
    const int rot = dev.pin_next++;
    const int b = rot % Device::kPinBufs, ci = rot & 1;
    hipStream_t cs = dev.pstream[ci];
    used[ci] = true;
    const uint32_t k = sizes[t];
    // buffer b is free once the last batch that used it (this call's or another's) is done
    HIPCHK(ctx, hipStreamWaitEvent(xs, dev.pin_free[b], 0));
    const uint8_t* src_pk = pk ? pk + 32 * i : (const uint8_t*)(key_idx + i);
    const std::vector<uint32_t> cut = schedule(t == 0, k);
    std::vector<uint32_t> marks;  // chunk ends, signatures
    for (uint32_t c = 0; c + 1 < cut.size() && cut[c] < k; c++) {
      const uint32_t o = cut[c];
      const size_t r = std::min(cut[c + 1], k) - o;
      marks.push_back(o + (uint32_t)r);
      HIPCHK(ctx, hipMemcpyAsync(dev.pin_msg[b].as<uint8_t>() + 32 * (size_t)o, msg + 32 * (i + o), 32 * r,
                                 hipMemcpyHostToDevice, xs));
      HIPCHK(ctx, hipMemcpyAsync(dev.pin_sig[b].as<uint8_t>() + 64 * (size_t)o, sig + 64 * (i + o), 64 * r,
                                 hipMemcpyHostToDevice, xs));
      HIPCHK(ctx, hipMemcpyAsync(dev.pin_pk[b].as<uint8_t>() + kb * o, src_pk + kb * o, kb * r,
                                 hipMemcpyHostToDevice, xs));
      HIPCHK(ctx, hipEventRecord(dev.chunk_ev[b][c], xs));
    }
    // every chunk's prep on cs (a second prep stream per compute stream measured slower:
    // 163-167 vs 175-180 M/s; more streams than the 4 hardware queues share queues)
    const mvk::ChunkGate gate{dev.chunk_ev[b], (uint32_t)marks.size(), marks.data()};
    mv_status rc = enqueue_batch(ctx, dev, dev.pin_msg[b].as<uint8_t>(), dev.pin_sig[b].as<uint8_t>(),
                                 pk ? dev.pin_pk[b].as<uint8_t>() : dev.committee_pk.as<uint8_t>(),
                                 pk ? nullptr : dev.pin_pk[b].as<uint32_t>(), k, dev.pin_st[b].as<uint8_t>(), cs,
                                 nullptr, &gate);
    hipError_t e = rc == MV_OK ? hipMemcpyAsync(hst + (i - lo), dev.pin_st[b].p, k, hipMemcpyDeviceToHost, cs)
                               : hipSuccess;
    if (e == hipSuccess && rc == MV_OK) e = hipEventRecord(dev.pin_free[b], cs);
    if (rc != MV_OK || e != hipSuccess) {
      // drain what was queued (it reads the input buffers and writes h_out) before returning
      (void)hipStreamSynchronize(xs);
      (void)hipStreamSynchronize(dev.pstream[0]);
      (void)hipStreamSynchronize(dev.pstream[1]);
      if (rc != MV_OK) return rc;
      return set_err(ctx, MV_E_HIP, std::string("streamed verify: ") + hipGetErrorString(e));
    }
  }
  for (int k = 0; k < 2; k++) HIPCHK(ctx, hipEventRecord(dev.sig_done[slot][k], dev.pstream[used[k] ? k : 1 - k]));
  return MV_OK;
}

}  // namespace

// ---- runtime switches (mvk::Knobs) -------------------------------------------
// Read from the environment once, at mv_create -- as the reference reads its knobs at start-up
// (validator.rs:104-119, config.rs:39-100) -- never per call: a multi-threaded host may call
// setenv, and getenv racing it is undefined behaviour. mv_set_option changes one afterwards.
namespace {
enum KnobKind { K_ON, K_OFF, K_FLAG, K_INT };  // on unless "0..." | on iff "1..." | on if set | integer
struct KnobDef {
  const char* name;
  int64_t mvk::Knobs::*field;
  KnobKind kind;
  bool create_only;  // consumed by mv_create: mv_set_option refuses it
};
const KnobDef kKnobs[] = {
    {"MV_BLK_PIPE", &mvk::Knobs::blk_pipe, K_ON, false},
    {"MV_COMB_SPLIT_BYTES", &mvk::Knobs::comb_split_bytes, K_INT, false},
    {"MV_HASH_IN_COMB", &mvk::Knobs::hash_in_comb, K_ON, false},
    {"MV_INGEST_IN_COMB", &mvk::Knobs::ingest_in_comb, K_ON, false},
    {"MV_VERDICT_FUSED", &mvk::Knobs::verdict_fused, K_ON, false},
    {"MV_BLK_CHUNK_BYTES", &mvk::Knobs::blk_chunk_bytes, K_INT, false},
    {"MV_PACK_THREADS", &mvk::Knobs::pack_threads, K_INT, false},
    {"MV_BLK_TRACE", &mvk::Knobs::blk_trace, K_FLAG, false},
    {"MV_BLK_ZEROCOPY", &mvk::Knobs::blk_zerocopy, K_INT, false},
    {"MV_PASS_SPIN", &mvk::Knobs::pass_spin, K_OFF, false},
    {"MV_PASS_SETS", &mvk::Knobs::pass_sets, K_INT, true},
    {"MV_Q_LINGER_US", &mvk::Knobs::q_linger_us, K_INT, false},
    {"MV_Q_SPIN_US", &mvk::Knobs::q_spin_us, K_INT, false},
    {"MV_ONLINE", &mvk::Knobs::online, K_ON, false},
    {"MV_ONLINE_LONG", &mvk::Knobs::online_long, K_ON, false},
    {"MV_ONLINE_PRIO", &mvk::Knobs::online_prio, K_ON, false},
    {"MV_ONLINE_WGS", &mvk::Knobs::online_wgs, K_INT, false},
    {"MV_ONLINE_IDLE_US", &mvk::Knobs::online_idle_us, K_INT, false},
    {"MV_ONLINE_TRACE", &mvk::Knobs::online_trace, K_FLAG, false},
    {"MV_ONLINE_DEBUG", &mvk::Knobs::online_debug, K_FLAG, false},
    {"MV_ONLINE_INJECT", &mvk::Knobs::online_inject, K_OFF, false},
    {"MV_ONLINE_SPINNERS", &mvk::Knobs::online_spinners, K_INT, false},
    {"MV_STREAM_CHUNK_LOG2", &mvk::Knobs::stream_chunk_log2, K_INT, false},
    {"MV_GUARD_GROUPS", &mvk::Knobs::guard_groups, K_INT, true},
    {"MV_BASE_GROUPS", &mvk::Knobs::base_groups, K_INT, true},
    {"MV_NO_KEY_AGG", &mvk::Knobs::no_key_agg, K_OFF, false},
    {"MV_REDUCE_QUAD", &mvk::Knobs::reduce_quad, K_INT, false},
    {"MV_BV_SEG", &mvk::Knobs::bv_seg, K_INT, false},
    {"MV_B2Q_NS", &mvk::Knobs::b2q_ns, K_INT, false},
    {"MV_B2_LANE", &mvk::Knobs::b2_lane, K_ON, false},
    {"MV_COMB_QUAD", &mvk::Knobs::comb_quad, K_INT, false},
    {"MV_INGEST_LANE", &mvk::Knobs::ingest_lane, K_OFF, false},
    {"MV_VERIFY_OCC", &mvk::Knobs::verify_occ, K_INT, false},
    {"MV_PREP_CHAIN", &mvk::Knobs::prep_chain, K_INT, false},
    {"MV_BLK_WALK", &mvk::Knobs::blk_walk, K_ON, false},
    {"MV_BUCKET_BAL", &mvk::Knobs::bucket_bal, K_INT, false},
    {"MV_FINAL_ROWS", &mvk::Knobs::final_rows, K_ON, false},
    {"MV_SCATTER_LDS", &mvk::Knobs::scatter_lds, K_ON, false},
    {"MV_FINE_LDS", &mvk::Knobs::fine_lds, K_ON, false},
    {"MV_REDUCE_ROWS", &mvk::Knobs::reduce_rows, K_INT, false},
};

const KnobDef* find_knob(const char* name) {
  if (!name) return nullptr;
  for (const KnobDef& d : kKnobs)
    if (strcmp(d.name, name) == 0) return &d;
  return nullptr;
}

mvk::Knobs knobs_from_env() {
  mvk::Knobs k;
  for (const KnobDef& d : kKnobs) {
    const char* e = getenv(d.name);
    if (!e || (!*e && d.kind != K_FLAG)) continue;
    switch (d.kind) {
      case K_ON: k.*d.field = e[0] != '0'; break;
      case K_OFF: k.*d.field = e[0] == '1'; break;
      case K_FLAG: k.*d.field = 1; break;
      case K_INT: k.*d.field = atoll(e); break;
    }
  }
  if (const char* e = getenv("MV_STREAM_FRACS")) {  // shares separated by ',' or '/'
    int n = 0;
    std::string x = e;
    for (size_t q = 0; q < x.size() && n < 8;) {
      size_t c = x.find_first_of(",/", q);
      if (c == std::string::npos) c = x.size();
      const double f = atof(x.substr(q, c - q).c_str());
      if (f > 0.0) k.stream_fracs[n++] = f;
      q = c + 1;
    }
    if (n == 0) k.stream_fracs[n++] = 1.0;
    k.n_stream_fracs = n;
  }
  return k;
}
}  // namespace

extern "C" {

const char* mv_version(void) { return "mysti_verify 0.2 gfx950"; }

namespace {
// Frees the retired buffers of `dev` that no call in flight reads (reap_ready), unless the
// online service of its GPU is running (its kernel would hold the free's device drain). Called
// with ctx->mu held at the start of the calls that grow buffers; o.mu is held across the check
// and the frees, so no launch starts in between.
void reap_idle(mv_ctx* ctx, Device& dev) {
  if (g_retired_n.load(std::memory_order_relaxed) == 0) return;
  std::shared_ptr<OnlineSvc> o;
  for (Device& d : ctx->devs)
    if (d.id == dev.id && d.online) o = d.online;  // one service per GPU (the first logical shard's)
  if (!o) {
    reap_ready(dev.id);
    return;
  }
  std::lock_guard<std::mutex> lk(o->mu);
  if (o->stuck) return;
  if (o->launched) {
    const hipError_t q = hipEventQuery(o->exited);
    if (q != hipSuccess) {
      (void)hipGetLastError();  // running (hipErrorNotReady)
      return;
    }
  }
  reap_ready(dev.id);
}
}  // namespace

mv_status mv_host_alloc(mv_ctx* ctx, uint64_t bytes, void** out) {
  if (!ctx || !out) return set_err(ctx, MV_E_INVALID_ARG, "bad host_alloc args");
  *out = nullptr;
  if (bytes == 0) return MV_OK;
  HIPCHK(ctx, hipSetDevice(ctx->devs[0].id));
  if (hipHostMalloc(out, bytes, hipHostMallocPortable) != hipSuccess) {
    (void)hipGetLastError();
    *out = nullptr;
    return set_err(ctx, MV_E_ALLOC, "hipHostMalloc failed");
  }
  return MV_OK;
}

void mv_host_free(mv_ctx* ctx, void* p) {
  (void)ctx;
  if (p) (void)hipHostFree(p);
}

int64_t mv_block_preimage(const uint8_t* bincode, uint64_t len, uint8_t* out, uint64_t cap) {
  if (!bincode && len) return -1;
  mvh::BlockFacts f;
  if (!mvh::parse_block(bincode, len, nullptr, out, out ? cap : 0, f)) return -1;
  return (int64_t)f.preimage_len;
}


mv_status mv_set_option(mv_ctx* ctx, const char* name, int64_t value) {
  if (!ctx) return MV_E_INVALID_ARG;
  const KnobDef* d = find_knob(name);
  if (!d) return set_err(ctx, MV_E_INVALID_ARG, std::string("unknown option ") + (name ? name : "(null)"));
  if (d->create_only) return set_err(ctx, MV_E_INVALID_ARG, std::string(name) + " is read at mv_create only");
  std::lock_guard<std::mutex> lk(ctx->mu);
  ctx->kn.*d->field = d->kind == K_INT ? value : (value != 0);
  return MV_OK;
}

mv_status mv_get_option(mv_ctx* ctx, const char* name, int64_t* value) {
  if (!ctx || !value) return MV_E_INVALID_ARG;
  const KnobDef* d = find_knob(name);
  if (!d) return set_err(ctx, MV_E_INVALID_ARG, std::string("unknown option ") + (name ? name : "(null)"));
  *value = ctx->kn.*d->field;
  return MV_OK;
}

mv_status mv_create(const mv_config* cfg, mv_ctx** out) {
  if (!out) return MV_E_INVALID_ARG;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return MV_E_NO_DEVICE;
  uint32_t mask = cfg && cfg->device_mask ? cfg->device_mask : 1u;
  mv_ctx* ctx = new mv_ctx();
  if (cfg && cfg->max_batch) ctx->max_batch = cfg->max_batch;
  if (cfg) ctx->flags = cfg->flags;
  ctx->kn = knobs_from_env();  // the only environment read: every switch, once
  if (ctx->kn.guard_groups >= 1 && ctx->kn.guard_groups <= mvk::BATCH_MAX_GROUPS)  // sub-batches while guarded
    ctx->guard_groups = (uint32_t)ctx->kn.guard_groups;
  if (ctx->kn.base_groups >= 1 && ctx->kn.base_groups <= mvk::BATCH_MAX_GROUPS)  // sub-batches when not guarded
    ctx->base_groups = (uint32_t)ctx->kn.base_groups;
  // two passes in flight: four measured worse on 16 concurrent 1-block callers (68.0 k vs
  // 72.2 k blocks/s, p99 203 vs 146 us; profiles/r03/c5_pass_sets.txt)
  ctx->q_sets = 2;
  if (ctx->kn.pass_sets >= 2 && ctx->kn.pass_sets <= Device::kPassSets) ctx->q_sets = (int)ctx->kn.pass_sets;
  {
    FILE* f = fopen("/dev/urandom", "rb");
    size_t got = f ? fread(ctx->secret, 1, sizeof(ctx->secret), f) : 0;
    if (f) fclose(f);
    if (got != sizeof(ctx->secret)) {
      delete ctx;
      return MV_E_INVALID_ARG;  // no entropy source: refuse rather than use predictable z_i
    }
  }
  // shards_per_device > 1: several logical devices (stream + buffers each) per HIP device;
  // host-buffer calls shard across them as across GPUs (tests the sharding on one GPU)
  const uint32_t reps = cfg && cfg->shards_per_device > 1 ? (cfg->shards_per_device > 8 ? 8 : cfg->shards_per_device) : 1;
  for (int d = 0; d < 32; d++) {
    if (!(mask & (1u << d))) continue;
    if (d >= ndev) {
      delete ctx;
      return MV_E_NO_DEVICE;
    }
    for (uint32_t r = 0; r < reps; r++) {
      Device dev;
      dev.id = d;
      ctx->devs.push_back(dev);
    }
  }
  for (auto& dev : ctx->devs) {
    hipError_t e = hipSetDevice(dev.id);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&dev.stream, hipStreamNonBlocking);
    for (int k = 0; k < 2 && e == hipSuccess; k++) e = hipStreamCreateWithFlags(&dev.pstream[k], hipStreamNonBlocking);
    // every other stream the engine uses, now: the runtime spreads streams over its hardware
    // queues (GPU_MAX_HW_QUEUES) in creation order, and the online service's stream must be
    // created after all of them, or a stream made later can share its queue and wait behind the
    // resident kernel (test_online_service_does_not_block_other_streams)
    for (int k = 0; k < Device::kPassSets && e == hipSuccess; k++)
      e = hipStreamCreateWithFlags(&dev.qstream[k], hipStreamNonBlocking);
    for (int k = 0; k < Device::kPassSets && e == hipSuccess; k++)
      e = hipStreamCreateWithFlags(&dev.pset[k].aux.stream, hipStreamNonBlocking);
    for (int k = 0; k < Device::kBlkSlots && e == hipSuccess; k++)
      e = hipStreamCreateWithFlags(&dev.blk_aux[k].stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = dev.btab.ensure(mvk::btable_bytes());
    if (e == hipSuccess) e = mvk::launch_btable_init(dev.btab.p, dev.stream);
    if (e == hipSuccess) e = dev.combB.ensure(mvk::comb_table_bytes(1));
    if (e == hipSuccess) e = mvk::launch_comb_init(nullptr, 1, 0, dev.combB.p, nullptr, dev.stream);
    if (e == hipSuccess) e = hipStreamSynchronize(dev.stream);
    if (e != hipSuccess) {
      mv_destroy(ctx);
      return MV_E_HIP;
    }
  }
  for (size_t i = 0; i < ctx->devs.size(); i++)
    if (i == 0 || ctx->devs[i].id != ctx->devs[i - 1].id) ctx->online_devs.push_back(i);
  *out = ctx;
  return MV_OK;
}

// Names the step a teardown is in on stderr while it takes longer than 5 s (a stall in
// mv_destroy otherwise looks like a silent hang to whoever waits for the process).
class PhaseWatch {
 public:
  explicit PhaseWatch(const char* what) : what_(what), th_([this] { run(); }) {}
  ~PhaseWatch() {
    {
      std::lock_guard<std::mutex> lk(m_);
      done_ = true;
    }
    cv_.notify_all();
    th_.join();
  }
  void phase(const char* p) { phase_.store(p); }

 private:
  void run() {
    std::unique_lock<std::mutex> lk(m_);
    for (int s = 5; !cv_.wait_for(lk, std::chrono::seconds(5), [this] { return done_; }); s += 5) {
      fprintf(stderr, "[%s] still in '%s' after %d s\n", what_, phase_.load(), s);
      if (s == 5) dump_threads();
    }
  }
  // every thread's name, kernel wait channel and current system call (/proc/self/task): tells a
  // runtime wait on a GPU signal (ioctl) from one on a lock (futex)
  static void dump_threads() {
    DIR* d = opendir("/proc/self/task");
    if (!d) return;
    while (dirent* e = readdir(d)) {
      if (e->d_name[0] == '.') continue;
      char path[128], comm[64] = {0}, wchan[64] = {0}, sc[160] = {0};
      auto rd = [&](const char* f, char* out, size_t cap) {
        snprintf(path, sizeof path, "/proc/self/task/%s/%s", e->d_name, f);
        if (FILE* fp = fopen(path, "r")) {
          size_t k = fread(out, 1, cap - 1, fp);
          out[k] = 0;
          fclose(fp);
          for (char* c = out; *c; c++)
            if (*c == '\n') *c = ' ';
        }
      };
      rd("comm", comm, sizeof comm);
      rd("wchan", wchan, sizeof wchan);
      rd("syscall", sc, sizeof sc);
      fprintf(stderr, "  tid %s %s wchan=%s syscall=%s\n", e->d_name, comm, wchan, sc);
    }
    closedir(d);
  }
  const char* what_;
  std::atomic<const char*> phase_{"start"};
  std::mutex m_;
  std::condition_variable cv_;
  bool done_ = false;
  std::thread th_;
};

void mv_destroy(mv_ctx* ctx) {
  if (!ctx) return;
  PhaseWatch watch("mv_destroy");
  watch.phase("stage events");
  (void)mv_stage_times(ctx, nullptr, nullptr, 1);  // drain pending stage events
  bool stuck = false;
  {
    watch.phase("online service stop");
    std::unique_lock<std::shared_mutex> cl(ctx->com_mu);
    for (auto& dev : ctx->devs)
      if (dev.online) {
        std::lock_guard<std::mutex> ol(dev.online->mu);
        (void)hipSetDevice(dev.id);
        online_release(*dev.online);  // before the device drain below: the kernel would hold it
        stuck |= dev.online->stuck;
      }
  }
  if (stuck) {
    // a resident launch that would not end still reads the engine's buffers: freeing them (or a
    // device drain, which would wait for it) is unsafe, so the context is abandoned, not freed
    fprintf(stderr, "[mv_destroy] the online service did not stop: the context's device memory is leaked\n");
    return;
  }
  for (auto& dev : ctx->devs) {
    (void)hipSetDevice(dev.id);
    watch.phase("engine stream drain");
    if (dev.stream) (void)hipStreamSynchronize(dev.stream);
    watch.phase("device drain");
    (void)hipDeviceSynchronize();  // device-API calls may have run on the caller's streams
    watch.phase("retired buffers");
    reap_retired(dev.id);
    watch.phase("frees: device buffers");
    for (DevBuf* b : {&dev.btab, &dev.combB, &dev.scratch, &dev.msg, &dev.sig, &dev.pk, &dev.keyidx, &dev.status,
                      &dev.bytes, &dev.off, &dev.len, &dev.out2, &dev.committee_pk, &dev.stakes, &dev.combA,
                      &dev.keyok, &dev.wal_tab, &dev.wal_rec, &dev.wal_mcount, &dev.wal_mflag,
                      &dev.wal_moff, &dev.wal_ent, &dev.wal_ff, &dev.wal_img, &dev.wal_pos, &dev.wal_tag, &dev.wal_len,
                      &dev.wal_st})
      b->release();
    watch.phase("frees: slot scratch");
    for (int k = 0; k < Device::kSlots; k++)
      for (DevBuf* b : {&dev.bscr[k], &dev.vscr[k], &dev.sscr[k]}) b->release();
    watch.phase("frees: block scratch");
    for (DevBuf& b : dev.blk) b.release();
    watch.phase("frees: slot events");
    for (hipEvent_t ev : dev.slot_done)
      if (ev) (void)hipEventDestroy(ev);
    for (hipEvent_t ev : dev.flag_ev)
      if (ev) (void)hipEventDestroy(ev);
    for (hipEvent_t ev : dev.sscr_done)
      if (ev) (void)hipEventDestroy(ev);
    watch.phase("frees: pinned-input buffers");
    for (int k = 0; k < Device::kPinBufs; k++) {
      for (DevBuf* b : {&dev.pin_msg[k], &dev.pin_sig[k], &dev.pin_pk[k], &dev.pin_st[k]}) b->release();
      if (dev.pin_free[k]) (void)hipEventDestroy(dev.pin_free[k]);
      for (hipEvent_t ev : dev.chunk_ev[k])
        if (ev) (void)hipEventDestroy(ev);
    }
    if (dev.prep_chain) (void)hipEventDestroy(dev.prep_chain);
    for (int k = 0; k < 2; k++) {
      watch.phase("frees: copy stream");
      if (dev.pstream[k]) (void)hipStreamDestroy(dev.pstream[k]);
    }
    watch.phase("frees: host flag words");
    if (dev.h_flags) (void)hipHostFree(dev.h_flags);
    watch.phase("frees: block events, aux streams");
    for (hipEvent_t ev : dev.blk_done)
      if (ev) (void)hipEventDestroy(ev);
    auto drop_aux = [](Device::BlkAux& a) {
      for (hipEvent_t ev : a.ev)
        if (ev) (void)hipEventDestroy(ev);
      if (a.stream) (void)hipStreamDestroy(a.stream);
    };
    for (auto& a : dev.blk_aux) drop_aux(a);
    for (auto& ps : dev.pset) drop_aux(ps.aux);
    watch.phase("frees: host in/out");
    dev.h_in.release();
    dev.h_out.release();
    watch.phase("frees: pass sets");
    for (auto& ps : dev.pset) {
      ps.h_in.release();
      ps.h_out.release();
      ps.bytes.release();
      ps.out2.release();
      ps.scr.release();
      if (ps.done) (void)hipEventDestroy(ps.done);
    }
    watch.phase("frees: queue streams");
    for (hipStream_t st : dev.qstream)
      if (st) (void)hipStreamDestroy(st);
    watch.phase("frees: engine stream");
    if (dev.stream) (void)hipStreamDestroy(dev.stream);
  }
  watch.phase("context");
  delete ctx;
}

const char* mv_last_error(const mv_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

mv_status mv_set_committee(mv_ctx* ctx, const uint8_t* pks, const uint64_t* stakes, uint32_t n, uint64_t epoch,
                           uint8_t* key_ok) {
  if (!ctx || !pks || !stakes || n == 0 || n > 512) return set_err(ctx, MV_E_INVALID_ARG, "bad committee args");
  std::unique_lock<std::shared_mutex> cl(ctx->com_mu);  // no online request in flight
  std::lock_guard<std::mutex> lk(ctx->mu);
  for (auto& dev : ctx->devs)
    if (dev.online) {
      std::lock_guard<std::mutex> ol(dev.online->mu);
      (void)hipSetDevice(dev.id);
      if (!online_stop(*dev.online))  // the resident kernel reads the tables rebuilt below
        return set_err(ctx, MV_E_HIP, "online service: the resident kernel did not stop");
    }
  mvh::Committee c;
  c.pks.assign(pks, pks + 32 * (size_t)n);
  c.stakes.assign(stakes, stakes + n);
  c.epoch = epoch;
  uint64_t total = 0;
  for (uint32_t i = 0; i < n; i++) total += stakes[i];
  c.quorum_threshold = 2 * total / 3;
  // unpublish first: if a device step fails below, the context is left with no committee
  // (block calls then refuse with MV_E_NO_COMMITTEE) rather than host facts that disagree
  // with half-built device tables
  ctx->has_committee = false;
  for (auto& dev : ctx->devs) dev.committee_loaded = false;
  for (auto& dev : ctx->devs) {
    HIPCHK(ctx, hipSetDevice(dev.id));
    HIPCHK(ctx, hipDeviceSynchronize());  // earlier device-API work may still read the old tables
    reap_retired(dev.id);                 // (the service is stopped: the drain waits for no resident kernel)
    HIPCHK(ctx, dev.committee_pk.ensure(32 * (size_t)n));
    HIPCHK(ctx, dev.stakes.ensure(8 * (size_t)n));
    HIPCHK(ctx, dev.combA.ensure(mvk::comb_table_bytes(n)));
    HIPCHK(ctx, dev.keyok.ensure(n));
    HIPCHK(ctx, hipMemcpyAsync(dev.committee_pk.p, pks, 32 * (size_t)n, hipMemcpyHostToDevice, dev.stream));
    HIPCHK(ctx, hipMemcpyAsync(dev.stakes.p, stakes, 8 * (size_t)n, hipMemcpyHostToDevice, dev.stream));
    // VerificationKey::try_from once per key (ZIP-215 decode) and its comb table of -A
    HIPCHK(ctx, mvk::launch_comb_init(dev.committee_pk.as<uint8_t>(), n, 1, dev.combA.p, dev.keyok.as<uint8_t>(),
                                      dev.stream));
    HIPCHK(ctx, hipStreamSynchronize(dev.stream));
  }
  if (key_ok) {
    Device& dev = ctx->devs[0];
    HIPCHK(ctx, hipSetDevice(dev.id));
    HIPCHK(ctx, hipMemcpy(key_ok, dev.keyok.p, n, hipMemcpyDeviceToHost));
  }
  ctx->committee = std::move(c);
  for (auto& dev : ctx->devs) dev.committee_loaded = true;
  ctx->has_committee = true;
  return MV_OK;
}

mv_status mv_blake2b256(mv_ctx* ctx, const uint8_t* buf, const uint64_t* off, const uint64_t* len, uint32_t n,
                        uint8_t* out) {
  if (!ctx || (n && (!buf || !off || !len || !out))) return set_err(ctx, MV_E_INVALID_ARG, "bad blake2b args");
  std::lock_guard<std::mutex> lk(ctx->mu);
  return for_each_shard(ctx, n, [&](Device& dev, uint64_t lo, uint64_t hi) -> mv_status {
    HIPCHK(ctx, hipSetDevice(dev.id));
    uint64_t i = lo;
    while (i < hi) {
      // chunk by count and by staged bytes (<= 1 GiB)
      uint64_t j = i, bytes = 0;
      while (j < hi && j - i < ctx->max_batch && bytes < (1ull << 30)) bytes += (len[j++] + 15) & ~7ull;
      uint32_t m = (uint32_t)(j - i);
      HIPCHK(ctx, dev.h_in.ensure(bytes + 16 * (size_t)m + 64));
      uint8_t* st = dev.h_in.as<uint8_t>();
      std::vector<uint64_t> soff(m), slen(m);
      uint64_t pos = 0;
      for (uint32_t k = 0; k < m; k++) {
        soff[k] = pos;
        slen[k] = len[i + k];
        memcpy(st + pos, buf + off[i + k], slen[k]);
        memset(st + pos + slen[k], 0, 8);
        pos += (slen[k] + 15) & ~7ull;
      }
      HIPCHK(ctx, dev.bytes.ensure(pos + 64));
      HIPCHK(ctx, dev.off.ensure(8 * (size_t)m));
      HIPCHK(ctx, dev.len.ensure(8 * (size_t)m));
      HIPCHK(ctx, dev.out2.ensure(32 * (size_t)m));
      HIPCHK(ctx, hipMemcpyAsync(dev.bytes.p, st, pos, hipMemcpyHostToDevice, dev.stream));
      HIPCHK(ctx, hipMemcpyAsync(dev.off.p, soff.data(), 8 * (size_t)m, hipMemcpyHostToDevice, dev.stream));
      HIPCHK(ctx, hipMemcpyAsync(dev.len.p, slen.data(), 8 * (size_t)m, hipMemcpyHostToDevice, dev.stream));
      HIPCHK(ctx, mvk::launch_blake2b(ctx->kn, dev.bytes.as<uint8_t>(), dev.off.as<uint64_t>(), dev.len.as<uint64_t>(), m,
                                      dev.out2.as<uint8_t>(), dev.stream));
      HIPCHK(ctx, hipMemcpyAsync(out + 32 * i, dev.out2.p, 32 * (size_t)m, hipMemcpyDeviceToHost, dev.stream));
      HIPCHK(ctx, hipStreamSynchronize(dev.stream));
      i = j;
    }
    return MV_OK;
  });
}

mv_status mv_ed25519_verify(mv_ctx* ctx, const uint8_t* msg, const uint8_t* sig, const uint8_t* pk,
                            const uint32_t* key_idx, uint32_t n, uint8_t* status) {
  if (!ctx || (n && (!msg || !sig || !status || (!pk == !key_idx))))
    return set_err(ctx, MV_E_INVALID_ARG, "bad verify args: exactly one of pk / key_idx");
  std::unique_lock<std::mutex> lk(ctx->mu);
  if (key_idx) {
    if (!ctx->has_committee) return set_err(ctx, MV_E_NO_COMMITTEE, "key_idx given but no committee set");
    for (uint32_t i = 0; i < n; i++)
      if (key_idx[i] >= ctx->committee.size()) return set_err(ctx, MV_E_INVALID_ARG, "key_idx out of range");
  }
  const bool pinned = n && host_pinned(msg) && host_pinned(sig) && host_pinned(pk ? (const void*)pk : key_idx);
  for (Device& d : ctx->devs) {
    HIPCHK(ctx, hipSetDevice(d.id));
    reap_idle(ctx, d);
  }
  // Pinned inputs (mv_host_alloc) of a large call stream: chunked DMA copies gate k_bv_prep
  // chunk by chunk (verify_host_streamed). The enqueue holds ctx->mu; the wait for the verdicts
  // does not, so concurrent callers' calls overlap (one's copies beside another's MSM; the
  // reference verifies in one task per peer, net_sync.rs:214-221). (Pageable inputs: one direct
  // H2D per max_batch below; a chunked pack into pinned staging and k_bv_prep reading pinned
  // inputs over PCIe measured slower and were removed in round 6)
  const bool streamed = pinned && !(ctx->flags & MV_FLAG_NO_BATCH);
  if (streamed) {
    const size_t nd = ctx->devs.size();
    std::vector<uint64_t> cut(nd + 1);
    for (size_t d = 0; d <= nd; d++) cut[d] = nd == 1 || n < 2 * 256 ? (d ? n : 0) : (uint64_t)n * d / nd;
    bool big = true;
    for (size_t d = 0; d < nd; d++) big &= cut[d + 1] == cut[d] || cut[d + 1] - cut[d] > 8ull * MV_BATCH_MIN;
    if (big) {
      // one staging slot per device for this call (wait while another call holds them all)
      std::vector<int> slot(nd, -1);
      auto free_slot = [&](Device& d) {
        for (int k = 0; k < Device::kSigCalls; k++)
          if (!d.sig_busy[k]) return k;
        return -1;
      };
      ctx->sig_cv.wait(lk, [&] {
        for (Device& d : ctx->devs)
          if (free_slot(d) < 0) return false;
        return true;
      });
      for (size_t d = 0; d < nd; d++) {
        slot[d] = free_slot(ctx->devs[d]);
        ctx->devs[d].sig_busy[slot[d]] = true;
      }
      mv_status rc = for_each_cut(ctx, cut, [&](Device& dev, uint64_t lo, uint64_t hi) -> mv_status {
        HIPCHK(ctx, hipSetDevice(dev.id));
        return verify_host_streamed(ctx, dev, msg, sig, pk, key_idx, lo, hi, slot[&dev - ctx->devs.data()]);
      });
      lk.unlock();
      // wait for this call's batches alone (events, not stream drains: another caller's batches
      // may follow on the same streams), then copy the verdicts out
      std::vector<hipError_t> werr(nd, hipSuccess);
      for (size_t d = 0; d < nd; d++) {
        if (cut[d + 1] == cut[d]) continue;
        Device& dev = ctx->devs[d];
        (void)hipSetDevice(dev.id);
        for (int k = 0; k < 2 && werr[d] == hipSuccess; k++) werr[d] = hipEventSynchronize(dev.sig_done[slot[d]][k]);
        if (rc == MV_OK && werr[d] == hipSuccess)
          memcpy(status + cut[d], dev.sig_stage[slot[d]].p, cut[d + 1] - cut[d]);
      }
      lk.lock();
      for (size_t d = 0; d < nd; d++) {
        Device& dev = ctx->devs[d];
        if (rc != MV_OK || werr[d] != hipSuccess) {  // drain what was queued before the slot is reused
          (void)hipSetDevice(dev.id);
          (void)hipStreamSynchronize(dev.stream);
          for (hipStream_t ps : dev.pstream) (void)hipStreamSynchronize(ps);
        }
        dev.sig_busy[slot[d]] = false;
        if (cut[d + 1] > cut[d]) {
          (void)hipSetDevice(dev.id);
          poll_flags(ctx, dev);
        }
      }
      ctx->sig_cv.notify_all();
      if (rc != MV_OK) return rc;
      for (size_t d = 0; d < nd; d++)
        if (werr[d] != hipSuccess)
          return set_err(ctx, MV_E_HIP, std::string("streamed verify: ") + hipGetErrorString(werr[d]));
      return MV_OK;
    }
  }
  return for_each_shard(ctx, n, [&](Device& dev, uint64_t lo, uint64_t hi) -> mv_status {
    HIPCHK(ctx, hipSetDevice(dev.id));
    for (uint64_t i = lo; i < hi; i += ctx->max_batch) {
      uint32_t m = (uint32_t)std::min<uint64_t>(ctx->max_batch, hi - i);
      HIPCHK(ctx, dev.msg.ensure(32 * (size_t)m));
      HIPCHK(ctx, dev.sig.ensure(64 * (size_t)m));
      HIPCHK(ctx, dev.status.ensure(m));
      HIPCHK(ctx, hipMemcpyAsync(dev.msg.p, msg + 32 * i, 32 * (size_t)m, hipMemcpyHostToDevice, dev.stream));
      HIPCHK(ctx, hipMemcpyAsync(dev.sig.p, sig + 64 * i, 64 * (size_t)m, hipMemcpyHostToDevice, dev.stream));
      const uint8_t* dpk;
      const uint32_t* dki = nullptr;
      if (pk) {
        HIPCHK(ctx, dev.pk.ensure(32 * (size_t)m));
        HIPCHK(ctx, hipMemcpyAsync(dev.pk.p, pk + 32 * i, 32 * (size_t)m, hipMemcpyHostToDevice, dev.stream));
        dpk = dev.pk.as<uint8_t>();
      } else {
        HIPCHK(ctx, dev.keyidx.ensure(4 * (size_t)m));
        HIPCHK(ctx, hipMemcpyAsync(dev.keyidx.p, key_idx + i, 4 * (size_t)m, hipMemcpyHostToDevice, dev.stream));
        dpk = dev.committee_pk.as<uint8_t>();
        dki = dev.keyidx.as<uint32_t>();
      }
      if (!(ctx->flags & MV_FLAG_NO_BATCH) && m >= MV_BATCH_MIN) {
        mv_status st = enqueue_batch(ctx, dev, dev.msg.as<uint8_t>(), dev.sig.as<uint8_t>(), dpk, dki, m,
                                     dev.status.as<uint8_t>(), dev.stream, nullptr);
        if (st != MV_OK) return st;
      } else if (dki) {
        mv_status st = enqueue_committee_verify(ctx, dev, dev.msg.as<uint8_t>(), dev.sig.as<uint8_t>(), dki, m,
                                                dev.status.as<uint8_t>(), dev.stream);
        if (st != MV_OK) return st;
      } else {
        mv_status st = enqueue_verify(ctx, dev, dev.msg.as<uint8_t>(), dev.sig.as<uint8_t>(), dpk, nullptr, m,
                                      dev.status.as<uint8_t>(), dev.stream);
        if (st != MV_OK) return st;
      }
      HIPCHK(ctx, hipMemcpyAsync(status + i, dev.status.p, m, hipMemcpyDeviceToHost, dev.stream));
      HIPCHK(ctx, hipStreamSynchronize(dev.stream));
      poll_flags(ctx, dev);
    }
    return MV_OK;
  });
}

mv_status mv_ed25519_sign(mv_ctx* ctx, const uint8_t* seed, const uint8_t* msg, uint32_t n, uint8_t* pk,
                          uint8_t* sig) {
  if (!ctx || (n && (!seed || !msg || !pk || !sig))) return set_err(ctx, MV_E_INVALID_ARG, "bad sign args");
  std::lock_guard<std::mutex> lk(ctx->mu);
  return for_each_shard(ctx, n, [&](Device& dev, uint64_t lo, uint64_t hi) -> mv_status {
    HIPCHK(ctx, hipSetDevice(dev.id));
    for (uint64_t i = lo; i < hi; i += ctx->max_batch) {
      uint32_t m = (uint32_t)std::min<uint64_t>(ctx->max_batch, hi - i);
      HIPCHK(ctx, dev.msg.ensure(32 * (size_t)m));
      HIPCHK(ctx, dev.bytes.ensure(32 * (size_t)m));
      HIPCHK(ctx, dev.pk.ensure(32 * (size_t)m));
      HIPCHK(ctx, dev.sig.ensure(64 * (size_t)m));
      HIPCHK(ctx, hipMemcpyAsync(dev.bytes.p, seed + 32 * i, 32 * (size_t)m, hipMemcpyHostToDevice, dev.stream));
      HIPCHK(ctx, hipMemcpyAsync(dev.msg.p, msg + 32 * i, 32 * (size_t)m, hipMemcpyHostToDevice, dev.stream));
      HIPCHK(ctx, mvk::launch_sign(dev.bytes.as<uint8_t>(), dev.msg.as<uint8_t>(), m, dev.btab.p,
                                   dev.pk.as<uint8_t>(), dev.sig.as<uint8_t>(), dev.stream));
      HIPCHK(ctx, hipMemcpyAsync(pk + 32 * i, dev.pk.p, 32 * (size_t)m, hipMemcpyDeviceToHost, dev.stream));
      HIPCHK(ctx, hipMemcpyAsync(sig + 64 * i, dev.sig.p, 64 * (size_t)m, hipMemcpyDeviceToHost, dev.stream));
      HIPCHK(ctx, hipStreamSynchronize(dev.stream));
    }
    return MV_OK;
  });
}

mv_status mv_verify_blocks(mv_ctx* ctx, const uint8_t* buf, const uint64_t* off, const uint64_t* len, uint32_t n,
                           uint8_t* status, uint8_t* msg_digest, uint8_t* block_digest) {
  if (!ctx || (n && (!buf || !off || !len || !status))) return set_err(ctx, MV_E_INVALID_ARG, "bad block args");
  if (!ctx->has_committee) {
    // a committee change in progress holds com_mu: wait for it rather than fail the call
    std::shared_lock<std::shared_mutex> cl(ctx->com_mu);
    if (!ctx->has_committee) return set_err(ctx, MV_E_NO_COMMITTEE, "mv_set_committee first");
  }
  if (n == 0) return MV_OK;
  if (ctx->flags & MV_FLAG_HOST_PARSE) {
    std::lock_guard<std::mutex> lk(ctx->mu);
    return verify_blocks_host_parse(ctx, buf, off, len, n, status, msg_digest, block_digest);
  }
  // the resident online service: small calls, no queue, no launch
  {
    uint64_t bytes = 0, longest = 0;
    for (uint32_t k = 0; k < n && bytes <= (128u << 10); k++) {
      bytes += (len[k] + 7) & ~7ull;
      longest = std::max<uint64_t>(longest, len[k]);
    }
    if (online_eligible(ctx, n, bytes, longest)) {
      std::shared_lock<std::shared_mutex> cl(ctx->com_mu);
      if (committee_ready(ctx)) {
        // one service per physical GPU: logical shards of one device (shards_per_device) share
        // the first shard's, so there is one resident kernel per GPU, not one per shard
        Device& dev = ctx->devs[ctx->online_devs[ctx->online_rr.fetch_add(1) % ctx->online_devs.size()]];
        {
          std::lock_guard<std::mutex> lk(ctx->mu);  // the service object (devs is fixed after mv_create)
          if (!dev.online) dev.online = std::make_shared<OnlineSvc>();
        }
        if (dev.online->failed) goto queue_path;  // a failed service: the submission queue serves
        std::string err;
        t_err = &err;
        const mv_status rc = online_verify(ctx, dev, buf, off, len, n, status, msg_digest, block_digest);
        t_err = nullptr;
        if (rc != MV_OK) {
          std::lock_guard<std::mutex> lk(ctx->mu);
          ctx->err = err;
        }
        return rc;
      }
    }
  }
queue_path:
  // Flat combining, pipelined: the request joins the queue; a caller that finds no pass being
  // packed and a free pass set takes every queued request (its own included) into one pass,
  // packs and enqueues it, then lets the next caller pack the following pass into the other
  // set while its own runs on the device. n - 1 peer tasks each submitting a block or two
  // (net_sync.rs:214-221, 314-386) thus share GPU round trips, up to q_sets passes in flight.
  mv_ctx::BlockReq req{buf, off, len, n, status, msg_digest, block_digest};
  ctx->q_calls++;
  const int linger_us = (int)ctx->kn.q_linger_us;  // MV_Q_LINGER_US, default 50 (profiles/r03/ab/queue_linger_*)
  // MV_Q_SPIN_US: a caller whose request is in another caller's pass polls for its verdicts
  // that long before sleeping on the queue's condition variable (no wake-up convoy on q_mu)
  const int spin_us = (int)ctx->kn.q_spin_us;
  bool lingered = false, spun = false;
  std::unique_lock<std::mutex> ql(ctx->q_mu);
  ctx->q.push_back(&req);
  if (ctx->q_lingering) ctx->q_linger_cv.notify_one();
  auto any_busy = [ctx] {
    for (int k = 0; k < ctx->q_sets; k++)
      if (ctx->q_set_busy[k]) return true;
    return false;
  };
  auto mark_all = [ctx](bool v) {
    for (int k = 0; k < ctx->q_sets; k++) ctx->q_set_busy[k] = v;
  };
  while (!req.done) {
    int s = -1;
    for (int k = 0; k < ctx->q_sets && s < 0; k++)
      if (!ctx->q_set_busy[k]) s = k;
    if (req.taken && spin_us > 0 && !spun) {
      spun = true;
      ql.unlock();
      const auto dl = std::chrono::steady_clock::now() + std::chrono::microseconds(spin_us);
      while (!req.done.load(std::memory_order_acquire) && std::chrono::steady_clock::now() < dl)
        std::this_thread::yield();
      ql.lock();
      continue;
    }
    if (ctx->q_packing || ctx->q_lingering || s < 0 || ctx->q.empty()) {
      ctx->q_cv.wait(ql);
      continue;
    }
    // Callers released together by a pass come back within microseconds of each other; the
    // first one back waits (bounded) for the others instead of starting a pass of one, so the
    // passes stay as large as the callers' groups (a lone caller's last pass carried 1: no wait)
    if (linger_us > 0 && !lingered && ctx->q.size() < ctx->q_last_calls) {
      lingered = true;
      ctx->q_lingering = true;
      const auto dl = std::chrono::steady_clock::now() + std::chrono::microseconds(linger_us);
      while (ctx->q.size() < ctx->q_last_calls && ctx->q_linger_cv.wait_until(ql, dl) != std::cv_status::timeout) {
      }
      ctx->q_lingering = false;
      ctx->q_cv.notify_all();
      continue;
    }
    std::deque<mv_ctx::BlockReq*> batch;
    batch.swap(ctx->q);  // no allocation
    for (auto* r : batch) r->taken = true;
    uint64_t blocks = 0, bytes = 0;
    for (auto* r : batch) {
      blocks += r->n;
      for (uint32_t k = 0; k < r->n; k++) bytes += (r->len[k] + 7) & ~7ull;
    }
    // larger than one chunk per device: the pass streams its chunks over both sets
    const uint64_t nd = ctx->devs.size();
    const bool big = blocks > (uint64_t)ctx->max_batch * nd || bytes > chunk_bytes_limit(ctx) * nd;
    ctx->q_packing = true;
    if (big)
      while (any_busy()) ctx->q_cv.wait(ql);
    const int set = big ? -1 : s;
    if (big) mark_all(true);
    else ctx->q_set_busy[s] = true;
    ql.unlock();
    run_block_requests(ctx, batch, set, [ctx] {
      std::lock_guard<std::mutex> lk(ctx->q_mu);
      ctx->q_packing = false;
      ctx->q_cv.notify_all();
    });
    ql.lock();
    ctx->q_last_calls = batch.size();
    for (auto* r : batch) r->done = true;
    if (big) mark_all(false);
    else ctx->q_set_busy[s] = false;
    ctx->q_cv.notify_all();
  }
  ql.unlock();
  if (req.rc != MV_OK) {
    std::lock_guard<std::mutex> lk(ctx->mu);
    ctx->err = req.err;
  }
  return req.rc;
}

mv_status mv_online_stats(mv_ctx* ctx, uint64_t* requests, uint64_t* launches) {
  if (!ctx) return MV_E_INVALID_ARG;
  uint64_t r = 0, l = 0;
  for (auto& dev : ctx->devs)
    if (dev.online) {
      r += dev.online->requests.load();
      l += dev.online->launches.load();
    }
  if (requests) *requests = r;
  if (launches) *launches = l;
  return MV_OK;
}

mv_status mv_queue_stats(mv_ctx* ctx, uint64_t* calls, uint64_t* passes) {
  if (!ctx) return MV_E_INVALID_ARG;
  if (calls) *calls = ctx->q_calls.load();
  if (passes) *passes = ctx->q_passes.load();
  return MV_OK;
}

mv_status mv_shard_plan(const uint64_t* weights, uint64_t n, uint32_t parts, uint64_t* cut) {
  if ((n && !weights) || !cut || parts == 0) return MV_E_INVALID_ARG;
  std::vector<uint64_t> c = balanced_cuts(weights, n, parts);
  memcpy(cut, c.data(), sizeof(uint64_t) * (parts + 1));
  return MV_OK;
}

static Device* find_dev(mv_ctx* ctx, int device) {
  for (auto& d : ctx->devs)
    if (d.id == device) return &d;
  return nullptr;
}

mv_status mv_dev_verify_blocks(mv_ctx* ctx, int device, const uint8_t* d_buf, uint64_t buf_bytes,
                               const uint64_t* d_off, const uint64_t* d_len, uint32_t n, uint8_t* d_status,
                               uint8_t* d_msg_digest, uint8_t* d_block_digest, void* stream) {
  if (!ctx || (n && (!d_buf || !d_off || !d_len || !d_status))) return set_err(ctx, MV_E_INVALID_ARG, "bad args");
  if (((uintptr_t)d_buf) & 7) return set_err(ctx, MV_E_INVALID_ARG, "d_buf must be 8-byte aligned");
  if ((((uintptr_t)d_msg_digest) | ((uintptr_t)d_block_digest)) & 15)
    return set_err(ctx, MV_E_INVALID_ARG, "digest arrays must be 16-byte aligned");
  std::lock_guard<std::mutex> lk(ctx->mu);
  if (!ctx->has_committee) return set_err(ctx, MV_E_NO_COMMITTEE, "mv_set_committee first");
  Device* dev = find_dev(ctx, device);
  if (!dev) return set_err(ctx, MV_E_NO_DEVICE, "device not in context");
  HIPCHK(ctx, hipSetDevice(dev->id));
  reap_idle(ctx, *dev);
  hipStream_t s = stream ? (hipStream_t)stream : dev->stream;
  return enqueue_blocks(ctx, *dev, d_buf, buf_bytes, d_off, d_len, n, d_status, d_msg_digest, d_block_digest, s);
}

mv_status mv_dev_ed25519_verify(mv_ctx* ctx, int device, const uint8_t* d_msg, const uint8_t* d_sig,
                                const uint8_t* d_pk, uint32_t n, uint8_t* d_status, void* stream) {
  if (!ctx || (n && (!d_msg || !d_sig || !d_pk || !d_status))) return set_err(ctx, MV_E_INVALID_ARG, "bad args");
  if ((((uintptr_t)d_msg) | ((uintptr_t)d_sig) | ((uintptr_t)d_pk)) & 15)
    return set_err(ctx, MV_E_INVALID_ARG, "device inputs must be 16-byte aligned");
  std::lock_guard<std::mutex> lk(ctx->mu);
  Device* dev = find_dev(ctx, device);
  if (!dev) return set_err(ctx, MV_E_NO_DEVICE, "device not in context");
  HIPCHK(ctx, hipSetDevice(dev->id));
  reap_idle(ctx, *dev);
  hipStream_t s = stream ? (hipStream_t)stream : dev->stream;
  return enqueue_verify(ctx, *dev, d_msg, d_sig, d_pk, nullptr, n, d_status, s);
}

mv_status mv_dev_ed25519_verify_batch(mv_ctx* ctx, int device, const uint8_t* d_msg, const uint8_t* d_sig,
                                      const uint8_t* d_pk, const uint32_t* d_key_idx, uint32_t n,
                                      uint8_t* d_status, uint32_t* d_batch_ok, void* stream) {
  if (!ctx || (n && (!d_msg || !d_sig || !d_pk || !d_status))) return set_err(ctx, MV_E_INVALID_ARG, "bad args");
  if ((((uintptr_t)d_msg) | ((uintptr_t)d_sig) | ((uintptr_t)d_pk)) & 15)
    return set_err(ctx, MV_E_INVALID_ARG, "device inputs must be 16-byte aligned");
  std::lock_guard<std::mutex> lk(ctx->mu);
  Device* dev = find_dev(ctx, device);
  if (!dev) return set_err(ctx, MV_E_NO_DEVICE, "device not in context");
  if (n == 0) return MV_OK;
  HIPCHK(ctx, hipSetDevice(dev->id));
  reap_idle(ctx, *dev);
  hipStream_t s = stream ? (hipStream_t)stream : dev->stream;
  return enqueue_batch(ctx, *dev, d_msg, d_sig, d_pk, d_key_idx, n, d_status, s, d_batch_ok, nullptr, true);
}

mv_status mv_batch_counters(mv_ctx* ctx, uint64_t* out) {
  if (!ctx || !out) return MV_E_INVALID_ARG;
  mv_status st = mv_batch_stats(ctx, out, out + 1);
  out[2] = ctx->groups_run.load();
  out[3] = ctx->groups_failed.load();
  return st;
}

mv_status mv_batch_routes(mv_ctx* ctx, uint64_t* out) {
  if (!ctx || !out) return MV_E_INVALID_ARG;
  mv_status st = mv_batch_stats(ctx, out, nullptr);  // accounts every completed batch first
  out[1] = ctx->single_batches.load();
  out[2] = ctx->dense_failures.load();
  return st;
}

mv_status mv_set_batch_groups(mv_ctx* ctx, uint32_t groups) {
  if (!ctx || groups > (uint32_t)mvk::BATCH_MAX_GROUPS) return set_err(ctx, MV_E_INVALID_ARG, "groups > 16");
  std::lock_guard<std::mutex> lk(ctx->mu);
  ctx->groups_fixed = groups;
  ctx->guard_left = 0;  // a new policy starts unguarded
  ctx->single_left = 0;
  return MV_OK;
}

mv_status mv_set_stage_timing(mv_ctx* ctx, int enable) {
  if (!ctx) return MV_E_INVALID_ARG;
  std::lock_guard<std::mutex> lk(ctx->mu);
  ctx->stage_timing = enable != 0;
  return MV_OK;
}

mv_status mv_stage_times(mv_ctx* ctx, double* ms, uint64_t* calls, int reset) {
  if (!ctx) return MV_E_INVALID_ARG;
  std::lock_guard<std::mutex> lk(ctx->tmu);
  for (auto& pe : ctx->pending) {
    HIPCHK(ctx, hipSetDevice(pe.device));
    std::vector<hipEvent_t>& ev = pe.events;
    HIPCHK(ctx, hipEventSynchronize(ev.back()));
    for (size_t i = 0; i + 1 < ev.size(); i++) {
      float t = 0;
      HIPCHK(ctx, hipEventElapsedTime(&t, ev[i], ev[i + 1]));
      ctx->stage_ms[pe.first_stage + i] += t;
      ctx->stage_calls[pe.first_stage + i]++;
    }
    for (hipEvent_t e : ev) (void)hipEventDestroy(e);
  }
  ctx->pending.clear();
  for (int i = 0; i < MV_NSTAGES; i++) {
    if (ms) ms[i] = ctx->stage_ms[i];
    if (calls) calls[i] = ctx->stage_calls[i];
  }
  if (reset) {
    for (double& x : ctx->stage_ms) x = 0;
    for (uint64_t& x : ctx->stage_calls) x = 0;
  }
  return MV_OK;
}

mv_status mv_batch_stats(mv_ctx* ctx, uint64_t* batches, uint64_t* fallbacks) {
  if (!ctx) return MV_E_INVALID_ARG;
  {
    std::lock_guard<std::mutex> lk(ctx->mu);
    for (auto& dev : ctx->devs) {
      (void)hipSetDevice(dev.id);
      poll_flags(ctx, dev);
    }
  }
  if (batches) *batches = ctx->batches.load();
  if (fallbacks) *fallbacks = ctx->fallbacks.load();
  return MV_OK;
}

mv_status mv_dev_ed25519_sign(mv_ctx* ctx, int device, const uint8_t* d_seed, const uint8_t* d_msg, uint32_t n,
                              uint8_t* d_pk, uint8_t* d_sig, void* stream) {
  if (!ctx || (n && (!d_seed || !d_msg || !d_pk || !d_sig))) return set_err(ctx, MV_E_INVALID_ARG, "bad args");
  if ((((uintptr_t)d_seed) | ((uintptr_t)d_msg) | ((uintptr_t)d_pk) | ((uintptr_t)d_sig)) & 15)
    return set_err(ctx, MV_E_INVALID_ARG, "device buffers must be 16-byte aligned");
  std::lock_guard<std::mutex> lk(ctx->mu);
  Device* dev = find_dev(ctx, device);
  if (!dev) return set_err(ctx, MV_E_NO_DEVICE, "device not in context");
  HIPCHK(ctx, hipSetDevice(dev->id));
  hipStream_t s = stream ? (hipStream_t)stream : dev->stream;
  HIPCHK(ctx, mvk::launch_sign(d_seed, d_msg, n, dev->btab.p, d_pk, d_sig, s));
  return MV_OK;
}

// ---------------------------------------------------------------- WAL replay
static mv_status wal_tables(mv_ctx* ctx, Device& dev) {
  if (dev.wal_tab.p) return MV_OK;
  std::vector<uint32_t> t(mvk::wal_table_words());
  mvk::wal_build_tables(t.data());
  HIPCHK(ctx, dev.wal_tab.ensure(4 * t.size()));
  HIPCHK(ctx, hipMemcpy(dev.wal_tab.p, t.data(), 4 * t.size(), hipMemcpyHostToDevice));
  if (!dev.cus) HIPCHK(ctx, hipDeviceGetAttribute(&dev.cus, hipDeviceAttributeMultiprocessorCount, dev.id));
  return MV_OK;
}

// Walk (one lane per map), join the maps in iteration order on the host, compact, crc pass.
static mv_status wal_run(mv_ctx* ctx, Device& dev, const uint8_t* d_img, uint64_t size, uint64_t end_pos,
                         uint32_t map_bits, uint64_t* d_pos, uint32_t* d_tag, uint32_t* d_len, uint8_t* d_status,
                         uint64_t cap, uint64_t* count, hipStream_t s) {
  *count = 0;
  mv_status st = wal_tables(ctx, dev);
  if (st != MV_OK) return st;
  const uint64_t msize = 1ull << map_bits, lim = std::min(size, end_pos);
  const uint64_t nmaps64 = (lim + msize - 1) >> map_bits;
  if (nmaps64 == 0) return MV_OK;
  if (nmaps64 > 0xffffffffull) return set_err(ctx, MV_E_INVALID_ARG, "too many maps");
  const uint32_t nmaps = (uint32_t)nmaps64;
  uint32_t cap_pm = (uint32_t)std::min<uint64_t>(msize / 16, 4096);
  std::vector<uint32_t> mcount(nmaps);
  std::vector<uint8_t> mflag(nmaps);
  uint32_t nincl = 0;
  uint64_t total = 0;
  std::vector<hipEvent_t> ew, ec;  // stage timing: walk, crc
  if ((st = make_events(ctx, 1, ew)) != MV_OK || (st = make_events(ctx, 1, ec)) != MV_OK) return st;
  auto mark = [&](std::vector<hipEvent_t>& e, int i) -> hipError_t {
    return e.empty() ? hipSuccess : hipEventRecord(e[i], s);
  };
  HIPCHK(ctx, dev.wal_rec.ensure(8 * (size_t)nmaps * cap_pm));
  HIPCHK(ctx, dev.wal_mcount.ensure(4 * (size_t)nmaps));
  HIPCHK(ctx, dev.wal_mflag.ensure(nmaps));
  HIPCHK(ctx, mark(ew, 0));
  HIPCHK(ctx, mvk::launch_wal_walk(d_img, size, end_pos, map_bits, nmaps, cap_pm, nullptr,
                                   dev.wal_rec.as<unsigned long long>(), dev.wal_mcount.as<uint32_t>(),
                                   dev.wal_mflag.as<uint8_t>(), s));
  HIPCHK(ctx, mark(ew, 1));
  HIPCHK(ctx, hipMemcpyAsync(mcount.data(), dev.wal_mcount.p, 4 * (size_t)nmaps, hipMemcpyDeviceToHost, s));
  HIPCHK(ctx, hipMemcpyAsync(mflag.data(), dev.wal_mflag.p, nmaps, hipMemcpyDeviceToHost, s));
  HIPCHK(ctx, hipStreamSynchronize(s));
  // WalIterator order: map after map while each one hands over to the next
  uint32_t maxc = 0;
  for (uint32_t m = 0; m < nmaps; m++) {
    if (mflag[m] == mvk::WAL_MAP_EMPTY) break;
    nincl = m + 1;
    total += mcount[m];
    maxc = std::max(maxc, mcount[m]);
    if (mflag[m] != mvk::WAL_MAP_NEXT) break;
  }
  keep_events(ctx, dev.id, kWalStage0, ew);
  if (total == 0) {
    for (hipEvent_t e : ec) (void)hipEventDestroy(e);
    return MV_OK;
  }
  std::vector<uint64_t> moff(nincl);
  for (uint64_t m = 0, o = 0; m < nincl; m++) {
    moff[m] = o;
    o += mcount[m];
  }
  HIPCHK(ctx, dev.wal_moff.ensure(8 * (size_t)nincl));
  HIPCHK(ctx, dev.wal_ent.ensure(8 * total));
  HIPCHK(ctx, dev.wal_ff.ensure(8));
  HIPCHK(ctx, hipMemcpyAsync(dev.wal_moff.p, moff.data(), 8 * (size_t)nincl, hipMemcpyHostToDevice, s));
  if (maxc <= cap_pm) {  // every map's records fit the first walk: compact them
    HIPCHK(ctx, mvk::launch_wal_compact(dev.wal_rec.as<unsigned long long>(), cap_pm, dev.wal_mcount.as<uint32_t>(),
                                        dev.wal_moff.as<uint64_t>(), nincl, dev.wal_ent.as<unsigned long long>(), s));
  } else {  // a map held more entries than the first guess: walk again straight into the entry list
    HIPCHK(ctx, mvk::launch_wal_walk(d_img, size, end_pos, map_bits, nincl, 0, dev.wal_moff.as<uint64_t>(),
                                     dev.wal_ent.as<unsigned long long>(), dev.wal_mcount.as<uint32_t>(),
                                     dev.wal_mflag.as<uint8_t>(), s));
  }
  HIPCHK(ctx, hipMemsetAsync(dev.wal_ff.p, 0xff, 8, s));
  HIPCHK(ctx, mark(ec, 0));
  HIPCHK(ctx, mvk::launch_wal_crc(d_img, size, dev.wal_ent.as<unsigned long long>(), total, dev.wal_tab.as<uint32_t>(),
                                  d_pos, d_tag, d_len, d_status, cap, dev.wal_ff.as<unsigned long long>(), dev.cus, s));
  HIPCHK(ctx, mark(ec, 1));
  keep_events(ctx, dev.id, kWalStage0 + 1, ec);
  uint64_t ff = 0;
  HIPCHK(ctx, hipMemcpyAsync(&ff, dev.wal_ff.p, 8, hipMemcpyDeviceToHost, s));
  HIPCHK(ctx, hipStreamSynchronize(s));
  *count = ff < total ? ff + 1 : total;
  return MV_OK;
}

static bool wal_args_ok(uint32_t map_bits) { return map_bits >= 8 && map_bits <= 30; }

mv_status mv_wal_verify(mv_ctx* ctx, const uint8_t* wal, uint64_t size, uint64_t end_pos, uint32_t map_bits,
                        uint64_t* pos, uint32_t* tag, uint32_t* len, uint8_t* status, uint64_t cap,
                        uint64_t* count) {
  if (!ctx || !count || (size && !wal) || (cap && (!pos || !tag || !len || !status)) || !wal_args_ok(map_bits))
    return set_err(ctx, MV_E_INVALID_ARG, "bad wal args");
  std::lock_guard<std::mutex> lk(ctx->mu);
  Device& dev = ctx->devs[0];  // one image, one device
  HIPCHK(ctx, hipSetDevice(dev.id));
  hipStream_t s = dev.stream;
  HIPCHK(ctx, dev.wal_img.ensure(size + 16));
  if (size) HIPCHK(ctx, hipMemcpyAsync(dev.wal_img.p, wal, size, hipMemcpyHostToDevice, s));
  // outputs: device arrays of up to cap entries; the walk bounds the entry count by size / 16
  const uint64_t ocap = std::min<uint64_t>(cap, size / 16 + 1);
  HIPCHK(ctx, dev.wal_pos.ensure(8 * ocap + 8));
  HIPCHK(ctx, dev.wal_tag.ensure(4 * ocap + 4));
  HIPCHK(ctx, dev.wal_len.ensure(4 * ocap + 4));
  HIPCHK(ctx, dev.wal_st.ensure(ocap + 1));
  uint64_t n = 0;
  mv_status st = wal_run(ctx, dev, dev.wal_img.as<uint8_t>(), size, end_pos, map_bits, dev.wal_pos.as<uint64_t>(),
                         dev.wal_tag.as<uint32_t>(), dev.wal_len.as<uint32_t>(), dev.wal_st.as<uint8_t>(), ocap, &n, s);
  if (st != MV_OK) return st;
  const uint64_t w = std::min(n, ocap);
  if (w) {
    HIPCHK(ctx, hipMemcpyAsync(pos, dev.wal_pos.p, 8 * w, hipMemcpyDeviceToHost, s));
    HIPCHK(ctx, hipMemcpyAsync(tag, dev.wal_tag.p, 4 * w, hipMemcpyDeviceToHost, s));
    HIPCHK(ctx, hipMemcpyAsync(len, dev.wal_len.p, 4 * w, hipMemcpyDeviceToHost, s));
    HIPCHK(ctx, hipMemcpyAsync(status, dev.wal_st.p, w, hipMemcpyDeviceToHost, s));
    HIPCHK(ctx, hipStreamSynchronize(s));
  }
  *count = n;
  return MV_OK;
}

mv_status mv_dev_wal_verify(mv_ctx* ctx, int device, const uint8_t* d_wal, uint64_t size, uint64_t end_pos,
                            uint32_t map_bits, uint64_t* d_pos, uint32_t* d_tag, uint32_t* d_len, uint8_t* d_status,
                            uint64_t cap, uint64_t* count, void* stream) {
  if (!ctx || !count || (size && !d_wal) || (cap && (!d_pos || !d_tag || !d_len || !d_status)) ||
      !wal_args_ok(map_bits))
    return set_err(ctx, MV_E_INVALID_ARG, "bad wal args");
  if (((uintptr_t)d_wal) & 3) return set_err(ctx, MV_E_INVALID_ARG, "d_wal must be 4-byte aligned");
  std::lock_guard<std::mutex> lk(ctx->mu);
  Device* dev = find_dev(ctx, device);
  if (!dev) return set_err(ctx, MV_E_NO_DEVICE, "device not in context");
  HIPCHK(ctx, hipSetDevice(dev->id));
  hipStream_t s = stream ? (hipStream_t)stream : dev->stream;
  return wal_run(ctx, *dev, d_wal, size, end_pos, map_bits, d_pos, d_tag, d_len, d_status, cap, count, s);
}

uint64_t mv_wal_layout(const uint64_t* payload_len, uint64_t n, uint32_t map_bits, uint64_t start, uint64_t* pos) {
  if (!wal_args_ok(map_bits) || (n && (!payload_len || !pos))) return start;
  const uint64_t mask = ~((1ull << map_bits) - 1);
  uint64_t p = start;
  for (uint64_t i = 0; i < n; i++) {
    const uint64_t len = payload_len[i] + 16;  // header + payload (wal.rs:152)
    if ((p & mask) != ((p + len - 1) & mask)) p = (p + len - 1) & mask;  // zero padding (wal.rs:163-167)
    pos[i] = p;
    p += len;
  }
  return p;
}

int64_t mv_frame_blocks(const uint8_t* buf, uint64_t len, uint64_t* off, uint64_t* blen, uint64_t cap,
                        uint64_t* consumed) {
  constexpr uint64_t kMaxSize = 16ull << 20;  // Network::MAX_SIZE (network.rs:216)
  constexpr uint64_t kPingRest = 8;           // PING_SIZE 12 - the size word (network.rs:425, 563)
  auto le = [&](uint64_t p, int bytes) {
    uint64_t v = 0;
    for (int k = 0; k < bytes; k++) v |= (uint64_t)buf[p + k] << (8 * k);
    return v;
  };
  if (consumed) *consumed = 0;
  if (len && !buf) return -1;
  if (cap && (!off || !blen)) return -1;
  uint64_t p = 0, found = 0;
  while (len - p >= 4) {
    const uint64_t size = ((uint64_t)buf[p] << 24) | ((uint64_t)buf[p + 1] << 16) | ((uint64_t)buf[p + 2] << 8) | buf[p + 3];
    if (size > kMaxSize) return -1;
    const uint64_t body = p + 4, need = size ? size : kPingRest;
    if (len - body < need) break;  // an incomplete frame: wait for more bytes
    const uint64_t end = body + need;
    if (size) {
      if (size < 4) return -1;  // no room for the message tag
      const uint64_t tag = le(body, 4);
      if (tag > 4) return -1;
      if (tag == 1 || tag == 3) {  // Blocks / RequestBlocksResponse: Vec<Data<StatementBlock>>
        if (end - body < 12) return -1;
        const uint64_t count = le(body + 4, 8);
        uint64_t q = body + 12;
        for (uint64_t k = 0; k < count; k++) {
          if (end - q < 8) return -1;
          const uint64_t l = le(q, 8);
          q += 8;
          if (l > end - q) return -1;
          if (found < cap) {
            off[found] = q;
            blen[found] = l;
          }
          found++;
          q += l;
        }
      }
    }
    p = end;
    if (consumed) *consumed = p;
  }
  return (int64_t)found;
}

mv_status mv_crc32(mv_ctx* ctx, const uint8_t* buf, const uint64_t* off, const uint64_t* len, uint32_t n,
                   uint32_t* out) {
  if (!ctx || (n && (!buf || !off || !len || !out))) return set_err(ctx, MV_E_INVALID_ARG, "bad crc32 args");
  std::lock_guard<std::mutex> lk(ctx->mu);
  return for_each_shard(ctx, n, [&](Device& dev, uint64_t lo, uint64_t hi) -> mv_status {
    HIPCHK(ctx, hipSetDevice(dev.id));
    mv_status st = wal_tables(ctx, dev);
    if (st != MV_OK) return st;
    uint64_t i = lo;
    while (i < hi) {
      uint64_t j = i, bytes = 0;  // chunks of <= max_batch strings and <= 1 GiB
      while (j < hi && j - i < ctx->max_batch && bytes < (1ull << 30)) bytes += len[j++];
      const uint32_t m = (uint32_t)(j - i);
      HIPCHK(ctx, dev.h_in.ensure(bytes + 16));
      uint8_t* stg = dev.h_in.as<uint8_t>();
      std::vector<uint64_t> soff(m), slen(m);
      uint64_t p = 0;
      for (uint32_t k = 0; k < m; k++) {
        soff[k] = p;
        slen[k] = len[i + k];
        memcpy(stg + p, buf + off[i + k], slen[k]);
        p += slen[k];
      }
      HIPCHK(ctx, dev.bytes.ensure(p + 16));
      HIPCHK(ctx, dev.off.ensure(8 * (size_t)m));
      HIPCHK(ctx, dev.len.ensure(8 * (size_t)m));
      HIPCHK(ctx, dev.out2.ensure(4 * (size_t)m));
      if (p) HIPCHK(ctx, hipMemcpyAsync(dev.bytes.p, stg, p, hipMemcpyHostToDevice, dev.stream));
      HIPCHK(ctx, hipMemcpyAsync(dev.off.p, soff.data(), 8 * (size_t)m, hipMemcpyHostToDevice, dev.stream));
      HIPCHK(ctx, hipMemcpyAsync(dev.len.p, slen.data(), 8 * (size_t)m, hipMemcpyHostToDevice, dev.stream));
      HIPCHK(ctx, mvk::launch_crc32(dev.bytes.as<uint8_t>(), dev.off.as<uint64_t>(), dev.len.as<uint64_t>(), m,
                                    dev.wal_tab.as<uint32_t>(), dev.out2.as<uint32_t>(), dev.cus, dev.stream));
      HIPCHK(ctx, hipMemcpyAsync(out + i, dev.out2.p, 4 * (size_t)m, hipMemcpyDeviceToHost, dev.stream));
      HIPCHK(ctx, hipStreamSynchronize(dev.stream));
      i = j;
    }
    return MV_OK;
  });
}

mv_status mv_dev_crc32(mv_ctx* ctx, int device, const uint8_t* d_buf, const uint64_t* d_off, const uint64_t* d_len,
                       uint32_t n, uint32_t* d_out, void* stream) {
  if (!ctx || (n && (!d_buf || !d_off || !d_len || !d_out))) return set_err(ctx, MV_E_INVALID_ARG, "bad args");
  if (((uintptr_t)d_buf) & 3) return set_err(ctx, MV_E_INVALID_ARG, "d_buf must be 4-byte aligned");
  std::lock_guard<std::mutex> lk(ctx->mu);
  Device* dev = find_dev(ctx, device);
  if (!dev) return set_err(ctx, MV_E_NO_DEVICE, "device not in context");
  HIPCHK(ctx, hipSetDevice(dev->id));
  mv_status st = wal_tables(ctx, *dev);
  if (st != MV_OK) return st;
  hipStream_t s = stream ? (hipStream_t)stream : dev->stream;
  HIPCHK(ctx, mvk::launch_crc32(d_buf, d_off, d_len, n, dev->wal_tab.as<uint32_t>(), d_out, dev->cus, s));
  return MV_OK;
}

mv_status mv_selftest(mv_ctx* ctx, int op, const uint32_t* in, uint32_t n, uint32_t* out) {
  if (!ctx || (n && (!in || !out))) return set_err(ctx, MV_E_INVALID_ARG, "bad selftest args");
  std::lock_guard<std::mutex> lk(ctx->mu);
  Device& dev = ctx->devs[0];
  HIPCHK(ctx, hipSetDevice(dev.id));
  HIPCHK(ctx, dev.bytes.ensure(64 * (size_t)n + 64));
  HIPCHK(ctx, dev.out2.ensure(64 * (size_t)n + 64));
  HIPCHK(ctx, hipMemcpyAsync(dev.bytes.p, in, 64 * (size_t)n, hipMemcpyHostToDevice, dev.stream));
  HIPCHK(ctx, mvk::launch_selftest(op, dev.bytes.as<uint32_t>(), n, dev.btab.p, dev.out2.as<uint32_t>(), dev.stream));
  HIPCHK(ctx, hipMemcpyAsync(out, dev.out2.p, 64 * (size_t)n, hipMemcpyDeviceToHost, dev.stream));
  HIPCHK(ctx, hipStreamSynchronize(dev.stream));
  return MV_OK;
}

}  // extern "C"
