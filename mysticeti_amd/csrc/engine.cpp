// libmysti_verify.so: contexts, device sharding and the C ABI of include/mysti_verify.h.
//
// One mv_ctx owns, per HIP device: a stream, the fixed-base table [0..128]B, and
// growable device / pinned-host buffers. Host-buffer calls split their items into
// one contiguous shard per device and run each shard on its own host thread
// (one stream per device, no collective: only per-item verdicts come back), in
// chunks of at most cfg.max_batch items. Calls on one ctx are serialised by a mutex.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/mysti_verify.h"
#include "block_codec.h"
#include "kernels.h"

namespace {

struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t bytes) {
    if (bytes <= cap) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    size_t want = std::max<size_t>(bytes, 4096);
    hipError_t e = hipMalloc(&p, want);
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
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
    size_t want = std::max<size_t>(bytes, 4096);
    hipError_t e = hipHostMalloc(&p, want, hipHostMallocDefault);
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

struct Device {
  int id = 0;
  hipStream_t stream = nullptr;
  DevBuf btab, scratch, msg, sig, pk, keyidx, status, bytes, off, len, out2, committee_pk;
  // batch-path scratch ring: consecutive batch calls alternate between two slots, so a
  // batch on one stream can run while the previous one (on another stream) finishes its
  // latency-bound tail; an event per slot orders reuse across streams
  static constexpr int kSlots = 2;
  DevBuf bscr[kSlots], vscr[kSlots];
  hipEvent_t slot_done[kSlots] = {nullptr, nullptr};
  bool slot_used[kSlots] = {false, false};
  int next_slot = 0;
  HostBuf h_in, h_out;
  bool committee_loaded = false;
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
  std::atomic<uint64_t> batches{0}, fallbacks{0};
  // batch-path stage timing (mv_set_stage_timing): event sets of calls not yet read back
  bool stage_timing = false;
  std::mutex tmu;
  std::vector<std::pair<int, std::vector<hipEvent_t>>> pending;  // (device, events)
  double stage_ms[mvk::BATCH_STAGES] = {0};
  uint64_t stage_calls = 0;
  bool has_committee = false;
  mvh::Committee committee;
};

namespace {

#define HIPCHK(ctx, expr)                                                                          \
  do {                                                                                             \
    hipError_t e_ = (expr);                                                                        \
    if (e_ != hipSuccess) {                                                                        \
      (ctx)->err = std::string(#expr) + ": " + hipGetErrorString(e_);                             \
      return MV_E_HIP;                                                                             \
    }                                                                                              \
  } while (0)

mv_status set_err(mv_ctx* ctx, mv_status code, const std::string& msg) {
  if (ctx) ctx->err = msg;
  return code;
}

// Runs fn(device, lo, hi) for each device's contiguous shard of [0, n), one thread per device.
template <class Fn>
mv_status for_each_shard(mv_ctx* ctx, uint64_t n, Fn fn) {
  const size_t nd = ctx->devs.size();
  if (nd == 1 || n < 2 * 256) {
    return fn(ctx->devs[0], 0, n);
  }
  std::vector<mv_status> rc(nd, MV_OK);
  std::vector<std::string> errs(nd);
  std::vector<std::thread> th;
  for (size_t d = 0; d < nd; d++) {
    uint64_t lo = n * d / nd, hi = n * (d + 1) / nd;
    th.emplace_back([&, d, lo, hi] {
      mv_status s = fn(ctx->devs[d], lo, hi);
      rc[d] = s;
    });
  }
  for (auto& t : th) t.join();
  for (size_t d = 0; d < nd; d++)
    if (rc[d] != MV_OK) return rc[d];
  return MV_OK;
}

// Enqueues the batch path (batch.hip) for n signatures on stream s.
mv_status enqueue_batch(mv_ctx* ctx, Device& dev, const uint8_t* d_msg, const uint8_t* d_sig, const uint8_t* d_pk,
                        const uint32_t* d_key_idx, uint32_t n, uint8_t* d_status, hipStream_t s, uint32_t* flag_dst,
                        bool flag_dst_host) {
  const int slot = dev.next_slot;
  dev.next_slot = (slot + 1) % Device::kSlots;
  if (!dev.slot_done[slot]) HIPCHK(ctx, hipEventCreateWithFlags(&dev.slot_done[slot], hipEventDisableTiming));
  if (dev.slot_used[slot]) HIPCHK(ctx, hipStreamWaitEvent(s, dev.slot_done[slot], 0));
  HIPCHK(ctx, dev.bscr[slot].ensure(mvk::batch_scratch_bytes(n)));
  HIPCHK(ctx, dev.vscr[slot].ensure(mvk::verify_scratch_bytes(n)));
  uint32_t key[10];
  memcpy(key, ctx->secret, 32);
  const uint64_t call = ctx->calls.fetch_add(1);
  key[8] = (uint32_t)call;
  key[9] = (uint32_t)(call >> 32);
  uint32_t* flag = nullptr;
  std::vector<hipEvent_t> evs;
  if (ctx->stage_timing) {
    evs.assign(mvk::BATCH_STAGES + 1, nullptr);
    for (auto& ev : evs) HIPCHK(ctx, hipEventCreate(&ev));
  }
  HIPCHK(ctx, mvk::launch_verify_batch(d_msg, d_sig, d_pk, d_key_idx, n, key, dev.btab.p, dev.bscr[slot].p,
                                       dev.vscr[slot].p, d_status, s, &flag, evs.empty() ? nullptr : evs.data()));
  if (!evs.empty()) {
    std::lock_guard<std::mutex> lk(ctx->tmu);
    ctx->pending.emplace_back(dev.id, std::move(evs));
  }
  if (flag_dst)
    HIPCHK(ctx, hipMemcpyAsync(flag_dst, flag, 4, flag_dst_host ? hipMemcpyDeviceToHost : hipMemcpyDeviceToDevice, s));
  HIPCHK(ctx, hipEventRecord(dev.slot_done[slot], s));
  dev.slot_used[slot] = true;
  return MV_OK;
}

}  // namespace

extern "C" {

const char* mv_version(void) { return "mysti_verify 0.1 gfx950"; }

int64_t mv_block_preimage(const uint8_t* bincode, uint64_t len, uint8_t* out, uint64_t cap) {
  if (!bincode && len) return -1;
  mvh::BlockFacts f;
  if (!mvh::parse_block(bincode, len, nullptr, out, out ? cap : 0, f)) return -1;
  return (int64_t)f.preimage_len;
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
  {
    FILE* f = fopen("/dev/urandom", "rb");
    size_t got = f ? fread(ctx->secret, 1, sizeof(ctx->secret), f) : 0;
    if (f) fclose(f);
    if (got != sizeof(ctx->secret)) {
      delete ctx;
      return MV_E_INVALID_ARG;  // no entropy source: refuse rather than use predictable z_i
    }
  }
  for (int d = 0; d < 32; d++) {
    if (!(mask & (1u << d))) continue;
    if (d >= ndev) {
      delete ctx;
      return MV_E_NO_DEVICE;
    }
    Device dev;
    dev.id = d;
    ctx->devs.push_back(dev);
  }
  for (auto& dev : ctx->devs) {
    hipError_t e = hipSetDevice(dev.id);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&dev.stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = dev.btab.ensure(mvk::btable_bytes());
    if (e == hipSuccess) e = mvk::launch_btable_init(dev.btab.p, dev.stream);
    if (e == hipSuccess) e = hipStreamSynchronize(dev.stream);
    if (e != hipSuccess) {
      mv_destroy(ctx);
      return MV_E_HIP;
    }
  }
  *out = ctx;
  return MV_OK;
}

void mv_destroy(mv_ctx* ctx) {
  if (!ctx) return;
  (void)mv_stage_times(ctx, nullptr, nullptr, 1);  // drain pending stage events
  for (auto& dev : ctx->devs) {
    (void)hipSetDevice(dev.id);
    if (dev.stream) (void)hipStreamSynchronize(dev.stream);
    for (DevBuf* b : {&dev.btab, &dev.scratch, &dev.msg, &dev.sig, &dev.pk, &dev.keyidx, &dev.status, &dev.bytes,
                      &dev.off, &dev.len, &dev.out2, &dev.committee_pk, &dev.bscr[0], &dev.bscr[1], &dev.vscr[0],
                      &dev.vscr[1]})
      b->release();
    for (hipEvent_t ev : dev.slot_done)
      if (ev) (void)hipEventDestroy(ev);
    dev.h_in.release();
    dev.h_out.release();
    if (dev.stream) (void)hipStreamDestroy(dev.stream);
  }
  delete ctx;
}

const char* mv_last_error(const mv_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

mv_status mv_set_committee(mv_ctx* ctx, const uint8_t* pks, const uint64_t* stakes, uint32_t n, uint64_t epoch,
                           uint8_t* key_ok) {
  if (!ctx || !pks || !stakes || n == 0 || n > 512) return set_err(ctx, MV_E_INVALID_ARG, "bad committee args");
  std::lock_guard<std::mutex> lk(ctx->mu);
  mvh::Committee c;
  c.pks.assign(pks, pks + 32 * (size_t)n);
  c.stakes.assign(stakes, stakes + n);
  c.epoch = epoch;
  uint64_t total = 0;
  for (uint32_t i = 0; i < n; i++) total += stakes[i];
  c.quorum_threshold = 2 * total / 3;
  ctx->committee = c;
  ctx->has_committee = true;
  for (auto& dev : ctx->devs) {
    HIPCHK(ctx, hipSetDevice(dev.id));
    HIPCHK(ctx, dev.committee_pk.ensure(32 * (size_t)n));
    HIPCHK(ctx, hipMemcpyAsync(dev.committee_pk.p, pks, 32 * (size_t)n, hipMemcpyHostToDevice, dev.stream));
    HIPCHK(ctx, hipStreamSynchronize(dev.stream));
    dev.committee_loaded = true;
  }
  if (key_ok) {
    // VerificationKey::try_from: ZIP-215 decode of each key (selftest op 7 on device 0)
    std::vector<uint32_t> in(16 * (size_t)n, 0), outw(16 * (size_t)n, 0);
    for (uint32_t i = 0; i < n; i++) memcpy(&in[16 * (size_t)i], pks + 32 * (size_t)i, 32);
    Device& dev = ctx->devs[0];
    HIPCHK(ctx, hipSetDevice(dev.id));
    HIPCHK(ctx, dev.bytes.ensure(in.size() * 4));
    HIPCHK(ctx, dev.out2.ensure(outw.size() * 4));
    HIPCHK(ctx, hipMemcpyAsync(dev.bytes.p, in.data(), in.size() * 4, hipMemcpyHostToDevice, dev.stream));
    HIPCHK(ctx, mvk::launch_selftest(7, dev.bytes.as<uint32_t>(), n, dev.btab.p, dev.out2.as<uint32_t>(), dev.stream));
    HIPCHK(ctx, hipMemcpyAsync(outw.data(), dev.out2.p, outw.size() * 4, hipMemcpyDeviceToHost, dev.stream));
    HIPCHK(ctx, hipStreamSynchronize(dev.stream));
    for (uint32_t i = 0; i < n; i++) key_ok[i] = outw[16 * (size_t)i + 8] ? 1 : 0;
  }
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
      HIPCHK(ctx, mvk::launch_blake2b(dev.bytes.as<uint8_t>(), dev.off.as<uint64_t>(), dev.len.as<uint64_t>(), m,
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
  std::lock_guard<std::mutex> lk(ctx->mu);
  if (key_idx) {
    if (!ctx->has_committee) return set_err(ctx, MV_E_NO_COMMITTEE, "key_idx given but no committee set");
    for (uint32_t i = 0; i < n; i++)
      if (key_idx[i] >= ctx->committee.size()) return set_err(ctx, MV_E_INVALID_ARG, "key_idx out of range");
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
      bool batched = false;
      uint32_t h_flag = 1;
      if (!(ctx->flags & MV_FLAG_NO_BATCH) && m >= MV_BATCH_MIN) {
        mv_status st = enqueue_batch(ctx, dev, dev.msg.as<uint8_t>(), dev.sig.as<uint8_t>(), dpk, dki, m,
                                     dev.status.as<uint8_t>(), dev.stream, &h_flag, true);
        if (st != MV_OK) return st;
        batched = true;
      } else {
        HIPCHK(ctx, dev.scratch.ensure(mvk::verify_scratch_bytes(m)));
        HIPCHK(ctx, mvk::launch_verify(dev.msg.as<uint8_t>(), dev.sig.as<uint8_t>(), dpk, dki, m, dev.btab.p,
                                       dev.scratch.p, dev.status.as<uint8_t>(), dev.stream));
      }
      HIPCHK(ctx, hipMemcpyAsync(status + i, dev.status.p, m, hipMemcpyDeviceToHost, dev.stream));
      HIPCHK(ctx, hipStreamSynchronize(dev.stream));
      if (batched) {
        ctx->batches++;
        if (!h_flag) ctx->fallbacks++;
      }
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
  std::lock_guard<std::mutex> lk(ctx->mu);
  if (!ctx->has_committee) return set_err(ctx, MV_E_NO_COMMITTEE, "mv_set_committee first");
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
      HIPCHK(ctx, mvk::launch_block_hash(dev.bytes.as<uint8_t>(), dev.off.as<uint64_t>(), dev.len.as<uint64_t>(), m,
                                         dev.msg.as<uint8_t>(), dev.out2.as<uint8_t>(), dev.stream));
      bool batched = false;
      uint32_t h_flag = 1;
      if (!(ctx->flags & MV_FLAG_NO_BATCH) && m >= MV_BATCH_MIN) {
        mv_status st = enqueue_batch(ctx, dev, dev.msg.as<uint8_t>(), dev.sig.as<uint8_t>(),
                                     dev.committee_pk.as<uint8_t>(), dev.keyidx.as<uint32_t>(), m,
                                     dev.status.as<uint8_t>(), dev.stream, &h_flag, true);
        if (st != MV_OK) return st;
        batched = true;
      } else {
        HIPCHK(ctx, dev.scratch.ensure(mvk::verify_scratch_bytes(m)));
        HIPCHK(ctx, mvk::launch_verify(dev.msg.as<uint8_t>(), dev.sig.as<uint8_t>(), dev.committee_pk.as<uint8_t>(),
                                       dev.keyidx.as<uint32_t>(), m, dev.btab.p, dev.scratch.p,
                                       dev.status.as<uint8_t>(), dev.stream));
      }
      std::vector<uint8_t> md(32 * (size_t)m), bd(32 * (size_t)m), ss(m);
      HIPCHK(ctx, hipMemcpyAsync(md.data(), dev.msg.p, 32 * (size_t)m, hipMemcpyDeviceToHost, dev.stream));
      HIPCHK(ctx, hipMemcpyAsync(bd.data(), dev.out2.p, 32 * (size_t)m, hipMemcpyDeviceToHost, dev.stream));
      HIPCHK(ctx, hipMemcpyAsync(ss.data(), dev.status.p, m, hipMemcpyDeviceToHost, dev.stream));
      HIPCHK(ctx, hipStreamSynchronize(dev.stream));
      if (batched) {
        ctx->batches++;
        if (!h_flag) ctx->fallbacks++;
      }
      for (uint32_t k = 0; k < m; k++) {
        status[i + k] = mvh::block_verdict(facts[k], com, &bd[32 * (size_t)k], ss[k]);
        if (msg_digest) memcpy(msg_digest + 32 * (i + k), &md[32 * (size_t)k], 32);
        if (block_digest) memcpy(block_digest + 32 * (i + k), &bd[32 * (size_t)k], 32);
      }
      i = j;
    }
    return MV_OK;
  });
}

static Device* find_dev(mv_ctx* ctx, int device) {
  for (auto& d : ctx->devs)
    if (d.id == device) return &d;
  return nullptr;
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
  hipStream_t s = stream ? (hipStream_t)stream : dev->stream;
  HIPCHK(ctx, dev->scratch.ensure(mvk::verify_scratch_bytes(n)));
  HIPCHK(ctx, mvk::launch_verify(d_msg, d_sig, d_pk, nullptr, n, dev->btab.p, dev->scratch.p, d_status, s));
  return MV_OK;
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
  hipStream_t s = stream ? (hipStream_t)stream : dev->stream;
  return enqueue_batch(ctx, *dev, d_msg, d_sig, d_pk, d_key_idx, n, d_status, s, d_batch_ok, false);
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
    HIPCHK(ctx, hipSetDevice(pe.first));
    std::vector<hipEvent_t>& ev = pe.second;
    HIPCHK(ctx, hipEventSynchronize(ev.back()));
    for (int i = 0; i < mvk::BATCH_STAGES; i++) {
      float t = 0;
      HIPCHK(ctx, hipEventElapsedTime(&t, ev[i], ev[i + 1]));
      ctx->stage_ms[i] += t;
    }
    for (hipEvent_t e : ev) (void)hipEventDestroy(e);
    ctx->stage_calls++;
  }
  ctx->pending.clear();
  if (ms)
    for (int i = 0; i < mvk::BATCH_STAGES; i++) ms[i] = ctx->stage_ms[i];
  if (calls) *calls = ctx->stage_calls;
  if (reset) {
    for (double& x : ctx->stage_ms) x = 0;
    ctx->stage_calls = 0;
  }
  return MV_OK;
}

mv_status mv_batch_stats(mv_ctx* ctx, uint64_t* batches, uint64_t* fallbacks) {
  if (!ctx) return MV_E_INVALID_ARG;
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
