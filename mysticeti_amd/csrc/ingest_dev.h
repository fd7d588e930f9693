// Device code of the block ingest, shared by ingest.hip's kernels and
// the online committee verify (comb.hip's k_verify_comb16, which ingests its own blocks). The
// rules and references are ingest.hip's header comment.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/mysti_verify.h"
#include "block_verdict.h"
#include "hash_dev.h"

namespace mv {

constexpr uint64_t VR_MAX_LEN = 1024 * 1024;  // VoteRange::verify MAX_LEN (types.rs:448)

// VoteRange::verify (types.rs:440-460), its checks in order: 1 = end < start, 2 = length
// >= MAX_LEN, 3 = end >= MAX_LEN, 0 = valid
MV_DEV uint32_t vr_code(uint64_t s0, uint64_t s1) {
  return s1 < s0 ? 1u : (s1 - s0 >= VR_MAX_LEN ? 2u : (s1 >= VR_MAX_LEN ? 3u : 0u));
}

// 8 little-endian bytes at any address (the buffer is readable 16 bytes past every block)
MV_DEV uint64_t peek8(const uint8_t* p) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  const uint64_t* w = reinterpret_cast<const uint64_t*>(a & ~static_cast<uintptr_t>(7));
  const uint32_t sh = static_cast<uint32_t>(a & 7u) * 8u;
  const uint64_t lo = w[0];
  return sh ? (lo >> sh) | (w[1] << (64u - sh)) : lo;
}

// bincode reader over one block; every read is checked against the block's length
struct BcReader {
  const uint8_t* p;
  uint64_t len, pos;
  bool ok;
  MV_DEV bool take(uint64_t k) {
    if (!ok || k > len - pos) ok = false;
    return ok;
  }
  MV_DEV uint64_t u64() {
    if (!take(8)) return 0;
    const uint64_t v = peek8(p + pos);
    pos += 8;
    return v;
  }
  MV_DEV uint32_t u32() {
    if (!take(4)) return 0;
    const uint32_t v = static_cast<uint32_t>(peek8(p + pos));
    pos += 4;
    return v;
  }
  MV_DEV uint32_t u8() {
    if (!take(1)) return 0;
    const uint32_t v = static_cast<uint32_t>(peek8(p + pos)) & 0xffu;
    pos += 1;
    return v;
  }
  // BlockReference: authority, round, digest (u64 length that must be 32, then 32 bytes)
  MV_DEV void ref(uint64_t& a, uint64_t& r, const uint8_t*& d) {
    a = u64();
    r = u64();
    const uint64_t l = u64();
    if (ok && l != 32) ok = false;
    d = p + pos;
    if (take(32)) pos += 32;
  }
};

// pre-image writer: bytes gathered into aligned 64-bit stores
struct PreWriter {
  uint64_t* out;
  uint64_t acc;
  uint32_t nb;  // bytes pending in acc (< 8)
  uint64_t len;
  // the k low bytes of v (1 <= k <= 8; the bytes of v above them are zero)
  MV_DEV void put(uint64_t v, uint32_t k) {
    acc |= v << (8 * nb);
    const uint32_t t = nb + k;
    if (t >= 8) {
      *out++ = acc;
      acc = nb ? v >> (64 - 8 * nb) : 0ull;
      nb = t - 8;
    } else {
      nb = t;
    }
    len += k;
  }
  MV_DEV void be64(uint64_t x) { put(__builtin_bswap64(x), 8); }
  MV_DEV void raw(const uint8_t* src, uint64_t k) {
    for (; k >= 8; k -= 8, src += 8) put(peek8(src), 8);
    if (k) put(peek8(src) & ((1ull << (8 * k)) - 1), static_cast<uint32_t>(k));
  }
  MV_DEV void ref(uint64_t a, uint64_t r, const uint8_t* d) {  // CryptoHash of BlockReference
    be64(a);
    be64(r);
    raw(d, 32);
  }
  MV_DEV void flush() {
    if (nb) *out++ = acc;
    acc = 0;
    nb = 0;
  }
};

// Outputs of the ingest of one block (all indexed by block).
struct IngestOut {
  uint8_t* stage;
  uint64_t* pre_off;
  uint64_t* pre_len;
  uint8_t* sig_out;
  uint32_t* key_idx;
  uint32_t* facts;
  uint8_t* claimed;
};
struct CommitteeView {
  const uint64_t* stakes;
  uint32_t n_auth;
  uint64_t epoch, quorum_thr;
};

// Block i = buf[o .. o + L), one lane, straight from global memory. P || sig (then 8 zero
// bytes) is written at stage + round_up(o, 8), which stays inside the block's own span
// because the bincode is at least |P| + 128 bytes long; writes happen only after the bytes
// they come from were read, so a malformed block never writes outside its span either.
// seen[k * stride], k < 16: a zeroed authority bitmap (<= 512 authorities) for this lane.
MV_DEV void ingest_lane(const uint8_t* buf, uint64_t o, uint64_t L, uint32_t i, const CommitteeView& cv,
                        const IngestOut& io, uint32_t* seen, int stride) {
  const uint32_t n_auth = cv.n_auth;
  const uint64_t so = (o + 7) & ~7ull;
  uint8_t* const stage = io.stage;
  BcReader r{buf + o, L, 0, true};
  PreWriter w{reinterpret_cast<uint64_t*>(stage + so), 0, 0, 0};

  uint64_t me_a, me_r;
  const uint8_t* me_d;
  r.ref(me_a, me_r, me_d);
  if (r.ok) {
    w.be64(me_a);
    w.be64(me_r);
  }
  // includes: pre-image, include checks (types.rs:349-362), threshold-clock stake
  const uint64_t n_inc = r.u64();
  uint32_t inc_err = 0;
  uint64_t stake = 0;
  bool quorum = false;
  for (uint64_t k = 0; r.ok && k < n_inc; k++) {
    uint64_t a, rd;
    const uint8_t* d;
    r.ref(a, rd, d);
    if (!r.ok) break;
    w.ref(a, rd, d);
    if (inc_err == 0) {
      if (a >= n_auth)
        inc_err = MV_BLOCK_INCLUDE_UNKNOWN_AUTHORITY;
      else if (rd >= me_r)
        inc_err = MV_BLOCK_INCLUDE_ROUND;
    }
    if (me_r > 0 && rd == me_r - 1 && a < n_auth) {
      const uint32_t wd = static_cast<uint32_t>(a) >> 5, bit = 1u << (a & 31);
      const uint32_t s = seen[wd * stride];
      if (!(s & bit)) {
        seen[wd * stride] = s | bit;
        stake += cv.stakes[a];
      }
      quorum = stake > cv.quorum_thr;
    }
  }
  // statements
  const uint64_t n_st = r.u64();
  uint32_t vr_first = 0;
  for (uint64_t k = 0; r.ok && k < n_st; k++) {
    const uint32_t tag = r.u32();
    if (!r.ok) break;
    if (tag == 0) {  // Share(Transaction): raw bytes, no length in the pre-image
      const uint64_t l = r.u64();
      if (!r.take(l)) break;
      w.put(0, 1);
      w.raw(r.p + r.pos, l);
      r.pos += l;
    } else if (tag == 1) {  // Vote(TransactionLocator, Vote)
      uint64_t a, rd;
      const uint8_t* d;
      r.ref(a, rd, d);
      const uint64_t lo = r.u64();
      const uint32_t vote = r.u32();
      if (!r.ok) break;
      if (vote == 0) {  // Accept
        w.put(1, 1);
        w.ref(a, rd, d);
        w.be64(lo);
      } else if (vote == 1) {  // Reject(Option<TransactionLocator>)
        const uint32_t some = r.u8();
        if (!r.ok) break;
        if (some == 0) {
          w.put(2, 1);
          w.ref(a, rd, d);
          w.be64(lo);
        } else if (some == 1) {
          uint64_t a2, rd2;
          const uint8_t* d2;
          r.ref(a2, rd2, d2);
          const uint64_t lo2 = r.u64();
          if (!r.ok) break;
          w.put(3, 1);
          w.ref(a, rd, d);
          w.be64(lo);
          w.ref(a2, rd2, d2);
          w.be64(lo2);
        } else {
          r.ok = false;
        }
      } else {
        r.ok = false;
      }
    } else if (tag == 2) {  // VoteRange(TransactionLocatorRange)
      uint64_t a, rd;
      const uint8_t* d;
      r.ref(a, rd, d);
      const uint64_t s0 = r.u64(), s1 = r.u64();
      if (!r.ok) break;
      w.put(4, 1);
      w.ref(a, rd, d);
      w.be64(s0);
      w.be64(s1);
      if (!vr_first) vr_first = vr_code(s0, s1);
    } else {
      r.ok = false;
    }
  }
  // meta_creation_time_ns (u128), epoch_marker (bool), epoch, signature
  const uint64_t tlo = r.u64(), thi = r.u64();
  const uint32_t marker = r.u8();
  if (r.ok && marker > 1) r.ok = false;
  const uint64_t ep = r.u64();
  const uint64_t sl = r.u64();
  if (r.ok && sl != 64) r.ok = false;
  const uint8_t* sp = r.p + r.pos;
  const bool parsed = r.take(64);
  uint32_t sw[16];
  uint32_t f = 0;
  if (parsed) {
    w.be64(thi);
    w.be64(tlo);
    w.put(marker, 1);
    w.be64(ep);
    const uint64_t plen = w.len;
#pragma unroll
    for (int q = 0; q < 8; q++) {
      const uint64_t v = peek8(sp + 8 * q);
      w.put(v, 8);
      sw[2 * q] = static_cast<uint32_t>(v);
      sw[2 * q + 1] = static_cast<uint32_t>(v >> 32);
    }
    w.put(0, 8);  // a zero word after P || sig
    w.flush();
    io.pre_len[i] = plen;
    f = BF_PARSED | (ep == cv.epoch ? BF_EPOCH_OK : 0u) | (me_a < n_auth ? BF_AUTHOR_OK : 0u) |
        (me_r == 0 ? BF_GENESIS : 0u) | (vr_first << BF_VR_SHIFT) | (quorum ? BF_QUORUM : 0u) |
        (inc_err << BF_INC_SHIFT);
    const uint64_t d0 = peek8(me_d), d1 = peek8(me_d + 8), d2 = peek8(me_d + 16), d3 = peek8(me_d + 24);
    uint4* cd = reinterpret_cast<uint4*>(io.claimed + 32 * (size_t)i);
    cd[0] = make_uint4((uint32_t)d0, (uint32_t)(d0 >> 32), (uint32_t)d1, (uint32_t)(d1 >> 32));
    cd[1] = make_uint4((uint32_t)d2, (uint32_t)(d2 >> 32), (uint32_t)d3, (uint32_t)(d3 >> 32));
  } else {
    io.pre_len[i] = 0;
#pragma unroll
    for (int q = 0; q < 16; q++) sw[q] = 0;
  }
  io.pre_off[i] = so;
  // a block rejected ahead of the signature check gets s = 2^256 - 1 (>= l): its verdict
  // does not depend on the signature, and s >= l keeps it out of the batch equation
  const bool sig_decides = parsed && (f & BF_EPOCH_OK) && (f & BF_AUTHOR_OK) && !(f & BF_GENESIS);
  if (!sig_decides) {
#pragma unroll
    for (int q = 8; q < 16; q++) sw[q] = 0xffffffffu;
  }
  uint4* so4 = reinterpret_cast<uint4*>(io.sig_out + 64 * (size_t)i);
#pragma unroll
  for (int q = 0; q < 4; q++) so4[q] = make_uint4(sw[4 * q], sw[4 * q + 1], sw[4 * q + 2], sw[4 * q + 3]);
  io.key_idx[i] = (parsed && me_a < n_auth) ? static_cast<uint32_t>(me_a) : 0u;
  io.facts[i] = f;
}

// ---------------------------------------------------------------- wave per block
// k_block_ingest: one 64-lane workgroup per block. The block's bincode is staged in LDS with
// coalesced 8-byte loads; the fixed-size includes are transcoded one per lane; the
// variable-size statements are located 64 at a time by lane 0 walking their headers, then
// transcoded one per lane (Share payloads copied by the whole wave); the pre-image is built
// in LDS and written to the stage with coalesced stores. Blocks that do not fit the LDS
// window take ingest_lane on lane 0. The rules are ingest_lane's (and block_codec.cpp's);
// tests/test_gpu_ingest.py holds the two kernels and the host codec to identical results.
constexpr uint32_t IG_WIN = 10240;  // LDS window per block, bytes
constexpr uint32_t IG_CHUNK = 64;   // statements located per walk

MV_DEV uint32_t lds_u8(const uint32_t* w, uint32_t p) { return (w[p >> 2] >> (8 * (p & 3))) & 0xffu; }
MV_DEV uint32_t lds_u32(const uint32_t* w, uint32_t p) {
  const uint32_t i = p >> 2, sh = (p & 3) * 8;
  return __builtin_amdgcn_alignbit(w[i + 1], w[i], sh);
}
MV_DEV uint64_t lds_u64(const uint32_t* w, uint32_t p) {
  const uint32_t i = p >> 2, sh = (p & 3) * 8;
  const uint32_t x0 = w[i], x1 = w[i + 1], x2 = w[i + 2];
  return ((uint64_t)__builtin_amdgcn_alignbit(x2, x1, sh) << 32) | __builtin_amdgcn_alignbit(x1, x0, sh);
}
MV_DEV void pre_be64(uint8_t* pre, uint32_t p, uint64_t x) {
#pragma unroll
  for (int b = 0; b < 8; b++) pre[p + b] = (uint8_t)(x >> (56 - 8 * b));
}
// 32 bytes of the window at byte q (any alignment): the 9 covering words, read together
MV_DEV void win_read32(uint32_t w[9], const uint32_t* win, uint32_t q) {
  const uint32_t i = q >> 2;
#pragma unroll
  for (int k = 0; k < 9; k++) w[k] = win[i + k];
}
// ... written to the pre-image at p (q = the byte address they were read from)
MV_DEV void pre_write32(uint8_t* pre, uint32_t p, const uint32_t w[9], uint32_t q) {
  const uint32_t sh = (q & 3) * 8;
#pragma unroll
  for (int k = 0; k < 8; k++) {
    const uint32_t x = __builtin_amdgcn_alignbit(w[k + 1], w[k], sh);
#pragma unroll
    for (int b = 0; b < 4; b++) pre[p + 4 * k + b] = (uint8_t)(x >> (8 * b));
  }
}
MV_DEV uint32_t wave_min(uint32_t x) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) x = min(x, (uint32_t)__shfl_xor((int)x, m));
  return x;
}
MV_DEV uint32_t wave_or(uint32_t x) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) x |= (uint32_t)__shfl_xor((int)x, m);
  return x;
}
MV_DEV uint64_t wave_sum64(uint64_t x) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
    const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)x, m), hi = (uint32_t)__shfl_xor((int)(uint32_t)(x >> 32), m);
    x += ((uint64_t)hi << 32) | lo;
  }
  return x;
}

// The LDS a wave needs to ingest one block.
struct IngestLds {
  uint64_t win64[IG_WIN / 8 + 4];
  uint32_t st_pos[IG_CHUNK], st_pre[IG_CHUNK];
  uint32_t seen[16];  // authorities of round r-1 among the includes
};
template <bool WAVE>
MV_DEV void ig_sync() {
  if (WAVE) {  // one wave of a larger workgroup (k_verify_comb16): wave-scope ordering
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  } else {
    __syncthreads();
  }
}

// Block i by one wave (k_block_ingest's body; WAVE: the wave is one of several in its
// workgroup and syncs alone). L: the wave's own LDS.
template <bool WAVE>
MV_DEV void ingest_block(uint32_t i, const uint8_t* __restrict__ buf, const uint64_t* __restrict__ off,
                         const uint64_t* __restrict__ len, const CommitteeView& cv, const IngestOut& io,
                         IngestLds& Ls) {
  uint64_t* win64 = Ls.win64;
  uint32_t* st_pos = Ls.st_pos;
  uint32_t* st_pre = Ls.st_pre;
  uint32_t* seen = Ls.seen;
  // The block's bincode (from its aligned start), transcoded IN PLACE into its pre-image ||
  // signature: every element's pre-image starts at or before its bincode and the elements
  // are produced in order, so an element's pre-image never reaches bincode not yet read
  // (each chunk's lanes read their elements into registers before any of them writes). One
  // 10-KB buffer instead of two doubles the waves per CU (LDS-limited, 7 -> 14).
  uint32_t* win = reinterpret_cast<uint32_t*>(win64);
  uint64_t* pre64 = win64;
  uint8_t* pre = reinterpret_cast<uint8_t*>(win64);
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t o = off[i], L = len[i];
  const uint32_t d = (uint32_t)(o & 7);
  if (lane < 16) seen[lane] = 0;
  if (d + L + 16 > IG_WIN) {  // does not fit the window: one lane from global memory
    ig_sync<WAVE>();
    if (lane == 0) ingest_lane(buf, o, L, i, cv, io, seen, 1);
    return;
  }
  {
    // every load of the window in flight at once (IG_LOADS per lane) before the LDS stores:
    // a store right behind each load would serialise the HBM latency 19 times for a 9.5-KB
    // block, and 16 per lane still took two rounds for it. The fit test above bounds nw by
    // IG_WIN / 8 = 64 * IG_LOADS, so one round always covers the block.
    constexpr int IG_LOADS = IG_WIN / 8 / 64;
    static_assert(IG_WIN % 512 == 0, "the window is whole 64-lane rounds of 8-byte loads");
    const uint64_t* src = reinterpret_cast<const uint64_t*>(buf + (o - d));
    uint64_t* w64 = win64;
    const uint32_t nw = (uint32_t)((d + L + 15) >> 3);
    uint64_t t[IG_LOADS];
#pragma unroll
    for (int j = 0; j < IG_LOADS; j++) t[j] = lane + 64 * j < nw ? src[lane + 64 * j] : 0ull;
#pragma unroll
    for (int j = 0; j < IG_LOADS; j++)
      if (lane + 64 * j < nw) w64[lane + 64 * j] = t[j];
  }
  ig_sync<WAVE>();
  const uint32_t Lb = (uint32_t)L;
  auto rd64 = [&](uint32_t p) { return lds_u64(win, d + p); };
  auto rd32 = [&](uint32_t p) { return lds_u32(win, d + p); };
  auto rd8 = [&](uint32_t p) { return lds_u8(win, d + p); };
  const uint32_t n_auth = cv.n_auth;

  // reference (56 B) and the include count
  bool ok = Lb >= 64;
  uint64_t me_a = 0, me_r = 0;
  if (ok) {
    me_a = rd64(0);
    me_r = rd64(8);
    ok = rd64(16) == 32;
  }
  const uint64_t n_inc = ok ? rd64(56) : 0;
  if (ok && n_inc > (uint64_t)((Lb - 64) / 56)) ok = false;
  // the claimed digest (bincode bytes 24..56), one word per lane 0..7, before the includes'
  // pre-images overwrite it
  const uint32_t claimed_w = (ok && lane < 8) ? rd32(24 + 4 * lane) : 0u;
  uint32_t bad = 0, inc_first = 0xffffffffu;
  if (ok) {
    if (lane < 8) {
      pre[lane] = (uint8_t)(me_a >> (56 - 8 * lane));
      pre[8 + lane] = (uint8_t)(me_r >> (56 - 8 * lane));
    }
    // includes: lane per include (pre-image at 16 + 48 k), checks (types.rs:349-362),
    // the threshold clock's authorities of round r-1 (threshold_clock.rs:12-35)
    for (uint32_t k = lane; k < (uint32_t)n_inc; k += 64) {
      const uint32_t p = 64 + 56 * k;
      const uint64_t a = rd64(p), r = rd64(p + 8);
      bad |= rd64(p + 16) != 32;
      uint64_t dg[4];
#pragma unroll
      for (int m = 0; m < 4; m++) dg[m] = rd64(p + 24 + 8 * m);  // digest bytes as they lie
      // pre-image offset 16 + 48 k is 8-byte aligned: six 64-bit LDS stores, not 48 byte stores
      uint64_t* pq = pre64 + 2 + 6 * k;
      pq[0] = __builtin_bswap64(a);  // big-endian u64 (pre_be64)
      pq[1] = __builtin_bswap64(r);
#pragma unroll
      for (int m = 0; m < 4; m++) pq[2 + m] = dg[m];
      const uint32_t code = a >= n_auth ? MV_BLOCK_INCLUDE_UNKNOWN_AUTHORITY : (r >= me_r ? MV_BLOCK_INCLUDE_ROUND : 0u);
      if (code && inc_first == 0xffffffffu) inc_first = (k << 4) | code;
      if (me_r > 0 && r == me_r - 1 && a < n_auth) atomicOr(&seen[(uint32_t)a >> 5], 1u << (a & 31));
    }
  }
  inc_first = wave_min(inc_first);
  // statements: located by lane 0 (headers only), 64 at a time, then transcoded per lane
  uint32_t pos = 64 + 56 * (uint32_t)n_inc, ppos = 16 + 48 * (uint32_t)n_inc;
  uint64_t n_st = 0;
  if (ok) {
    if (pos + 8 > Lb) ok = false;
    else n_st = rd64(pos);
    pos += 8;
  }
  uint32_t vr_first = 0xffffffffu;  // (statement index << 2) | vr_code of the first failing range
  for (uint64_t k0 = 0; ok && k0 < n_st; k0 += IG_CHUNK) {
    // Locate up to IG_CHUNK statements. Speculation: lane j assumes the j statements
    // before it are VoteRanges (76 B in bincode, 65 in the pre-image) and checks its own
    // tag; the run of confirmed VoteRanges is taken at once, anything else takes one
    // scalar step (the whole wave computes it identically).
    uint32_t c = 0, p = pos, pp = ppos;
    bool lok = true;
    while (c < IG_CHUNK && k0 + c < n_st) {
      const uint32_t j = c + lane;
      const uint32_t q = p + 76 * lane;
      const bool rng = j < IG_CHUNK && k0 + j < n_st && q + 76 <= Lb && rd32(q) == 2;
      const uint64_t brk = __ballot(!rng);
      const uint32_t run = brk ? (uint32_t)__builtin_ctzll(brk) : 64u;
      if (lane < run) {
        st_pos[j] = q;
        st_pre[j] = pp + 65 * lane;
      }
      c += run;
      p += 76 * run;
      pp += 65 * run;
      if (c >= IG_CHUNK || k0 + c >= n_st) break;
      uint32_t size = 0, psize = 0;
      if (p + 4 > Lb) { lok = false; break; }
      const uint32_t tag = rd32(p);
      if (tag == 0) {  // Share: u32 tag, u64 length, bytes
        if (p + 12 > Lb) { lok = false; break; }
        const uint64_t l = rd64(p + 4);
        if (l > (uint64_t)(Lb - p - 12)) { lok = false; break; }
        size = 12 + (uint32_t)l;
        psize = 1 + (uint32_t)l;
      } else if (tag == 1) {  // Vote: locator (64 B), u32 vote, [u8 option, [locator]]
        if (p + 72 > Lb) { lok = false; break; }
        const uint32_t vote = rd32(p + 68);
        if (vote == 0) {
          size = 72;
          psize = 57;
        } else if (vote == 1 && p + 73 <= Lb) {
          const uint32_t some = rd8(p + 72);
          if (some == 0) {
            size = 73;
            psize = 57;
          } else if (some == 1 && p + 137 <= Lb) {
            size = 137;
            psize = 113;
          } else {
            lok = false;
            break;
          }
        } else {
          lok = false;
          break;
        }
      } else {  // tag 2 here means a truncated VoteRange; others are invalid
        lok = false;
        break;
      }
      if (lane == 0) {
        st_pos[c] = p;
        st_pre[c] = pp;
      }
      c++;
      p += size;
      pp += psize;
    }
    ig_sync<WAVE>();
    const uint32_t cnt = c;
    ok = lok;
    // (a) every lane reads its statement into registers
    uint32_t kind = 0;  // 1 Share, 2 Accept, 3 Reject(None), 4 Reject(Some), 5 VoteRange
    uint32_t q = 0, ps = 0;
    uint64_t a = 0, r = 0, x = 0, y = 0, a2 = 0, r2 = 0, z2 = 0;
    uint32_t dg[9], dg2[9];
    if (lane < cnt) {
      const uint32_t p = st_pos[lane];
      q = st_pre[lane];
      ps = p;
      const uint32_t tag = rd32(p);
      if (tag == 0) {
        kind = 1;
      } else {
        a = rd64(p + 4);
        r = rd64(p + 12);
        bad |= rd64(p + 20) != 32;
        win_read32(dg, win, d + p + 28);
        x = rd64(p + 60);
        if (tag == 1) {
          const uint32_t vote = rd32(p + 68);
          const uint32_t some = vote == 1 ? rd8(p + 72) : 0u;
          kind = vote == 0 ? 2 : (some == 0 ? 3 : 4);
          if (kind == 4) {
            a2 = rd64(p + 73);
            r2 = rd64(p + 81);
            bad |= rd64(p + 89) != 32;
            win_read32(dg2, win, d + p + 97);
            z2 = rd64(p + 129);
          }
        } else {  // tag 2
          kind = 5;
          y = rd64(p + 68);
          const uint32_t code = vr_code(x, y);
          if (code && vr_first == 0xffffffffu) vr_first = ((uint32_t)(k0 + lane) << 2) | code;
        }
      }
    }
    // (b) Share payloads, moved down by the whole wave 64 bytes at a time (each round reads
    // before it writes, and the destination lies below the source)
    uint64_t shares = __ballot(kind == 1);
    while (shares) {
      const uint32_t j = (uint32_t)__builtin_ctzll(shares);
      shares &= shares - 1;
      const uint32_t p = st_pos[j], qj = st_pre[j];
      const uint32_t l = (uint32_t)rd64(p + 4);
      for (uint32_t t = lane; t < ((l + 63) & ~63u); t += 64) {
        const uint32_t v = t < l ? rd8(p + 12 + t) : 0u;
        if (t < l) pre[qj + 1 + t] = (uint8_t)v;
      }
    }
    // (c) every lane writes its statement's pre-image
    if (kind == 1) {
      pre[q] = 0;
    } else if (kind >= 2 && kind <= 4) {
      pre[q] = (uint8_t)(kind - 1);
      pre_be64(pre, q + 1, a);
      pre_be64(pre, q + 9, r);
      pre_write32(pre, q + 17, dg, d + ps + 28);
      pre_be64(pre, q + 49, x);
      if (kind == 4) {
        pre_be64(pre, q + 57, a2);
        pre_be64(pre, q + 65, r2);
        pre_write32(pre, q + 73, dg2, d + ps + 97);
        pre_be64(pre, q + 105, z2);
      }
    } else if (kind == 5) {
      pre[q] = 4;
      pre_be64(pre, q + 1, a);
      pre_be64(pre, q + 9, r);
      pre_write32(pre, q + 17, dg, d + ps + 28);
      pre_be64(pre, q + 49, x);
      pre_be64(pre, q + 57, y);
    }
    pos = p;
    ppos = pp;
    ig_sync<WAVE>();  // st_* are rewritten by the next chunk
  }
  // meta_creation_time_ns (u128 LE), epoch_marker (bool), epoch, signature (u64 64 + 64 B)
  uint64_t tlo = 0, thi = 0, ep = 0;
  uint32_t marker = 0;
  if (ok) {
    if (pos + 97 > Lb) {
      ok = false;
    } else {
      tlo = rd64(pos);
      thi = rd64(pos + 8);
      marker = rd8(pos + 16);
      ep = rd64(pos + 17);
      ok = marker <= 1 && rd64(pos + 25) == 64;
    }
  }
  ok = ok && wave_or(bad) == 0;
  const uint32_t spos = pos + 33;  // signature
  uint32_t f = 0;
  if (ok) {
    if (lane == 0) {
      pre_be64(pre, ppos, thi);
      pre_be64(pre, ppos + 8, tlo);
      pre[ppos + 16] = (uint8_t)marker;
      pre_be64(pre, ppos + 17, ep);
    }
    const uint32_t sb = rd8(spos + lane);  // P || sig (read by every lane before any writes)
    pre[ppos + 25 + lane] = (uint8_t)sb;
    // threshold clock: stake of the distinct round r-1 authorities among the includes
    // (lane j sums authorities j, j + 64, ...: independent loads, one latency)
    uint64_t stake = 0;
#pragma unroll
    for (uint32_t q = 0; q < 8; q++) {
      const uint32_t a = lane + 64 * q;
      if (a < n_auth && ((seen[a >> 5] >> (a & 31)) & 1u)) stake += cv.stakes[a];
    }
    stake = wave_sum64(stake);
    const uint32_t inc_code = inc_first == 0xffffffffu ? 0u : (inc_first & 15u);
    vr_first = wave_min(vr_first);
    const uint32_t vr = vr_first == 0xffffffffu ? 0u : (vr_first & 3u);
    f = BF_PARSED | (ep == cv.epoch ? BF_EPOCH_OK : 0u) | (me_a < n_auth ? BF_AUTHOR_OK : 0u) |
        (me_r == 0 ? BF_GENESIS : 0u) | (vr << BF_VR_SHIFT) | (stake > cv.quorum_thr ? BF_QUORUM : 0u) |
        (inc_code << BF_INC_SHIFT);
  }
  ig_sync<WAVE>();
  const uint64_t so = (o + 7) & ~7ull;
  const uint32_t plen = ppos + 25;
  if (ok) {  // P || sig to the stage (it stays inside the block's own span, see ingest_lane)
    uint64_t* dst = reinterpret_cast<uint64_t*>(io.stage + so);
    const uint32_t nw = (plen + 64 + 7) >> 3;
    for (uint32_t k = lane; k < nw; k += 64) dst[k] = pre64[k];
  }
  if (ok && lane < 8) reinterpret_cast<uint32_t*>(io.claimed + 32 * (size_t)i)[lane] = claimed_w;
  if (lane == 0) {
    io.pre_off[i] = so;
    io.pre_len[i] = ok ? plen : 0;
    uint32_t sw[16];  // the signature, from its pre-image copy (its bincode was overwritten)
#pragma unroll
    for (int q = 0; q < 16; q++) sw[q] = ok ? lds_u32(win, plen + 4 * q) : 0u;
    const bool sig_decides = ok && (f & BF_EPOCH_OK) && (f & BF_AUTHOR_OK) && !(f & BF_GENESIS);
    if (!sig_decides) {
#pragma unroll
      for (int q = 8; q < 16; q++) sw[q] = 0xffffffffu;
    }
    uint4* so4 = reinterpret_cast<uint4*>(io.sig_out + 64 * (size_t)i);
#pragma unroll
    for (int q = 0; q < 4; q++) so4[q] = make_uint4(sw[4 * q], sw[4 * q + 1], sw[4 * q + 2], sw[4 * q + 3]);
    io.key_idx[i] = (ok && me_a < n_auth) ? (uint32_t)me_a : 0u;
    io.facts[i] = f;
  }
}

}  // namespace mv
