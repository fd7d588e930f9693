// Device-side StatementBlock ingest for gfx950: bincode
// Data<StatementBlock> bytes resident in HBM -> the signed pre-image P || sig, staged for
// k_block_hash, plus the facts StatementBlock::verify checks; one block per lane.
// k_block_verdict folds the digest comparison, the signature verdict and those facts into
// one status in the reference's error order (types.rs:315-376).
//
//   bincode     types.rs:93-114 (StatementBlock), :49-54 (BlockReference), :57-64
//               (BaseStatement), :31-35 (Vote), :384-394 (locators), crypto.rs:309-347
//               (length-checked 32/64-byte arrays); bincode 1.3.3 defaults (LE fixint, u64
//               lengths, u32 tags, trailing bytes allowed) as Data::from_bytes uses them
//               (data.rs:43-52)
//   pre-image   BlockDigest::digest_without_signature (crypto.rs:85-128) with the
//               CryptoHash encodings of crypto.rs:150-170, types.rs:661-691 and 751-755
//   checks      epoch, author, genesis and includes (types.rs:333-362), VoteRange::verify
//               (types.rs:440-460), the threshold clock (threshold_clock.rs:12-35)
// block_codec.cpp states the same rules on the host (MV_FLAG_HOST_PARSE); the GPU tests hold
// both paths and the oracle to the same verdicts and digests, malformed input included.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/mysti_verify.h"
#include "hash_dev.h"
#include "kernels.h"

namespace mv {

constexpr uint32_t BF_PARSED = 1u, BF_EPOCH_OK = 2u, BF_AUTHOR_OK = 4u, BF_GENESIS = 8u, BF_VR_BAD = 16u,
                   BF_QUORUM = 32u;
constexpr int BF_INC_SHIFT = 8;               // first failing include: MV_BLOCK_INCLUDE_* or 0
constexpr uint64_t VR_MAX_LEN = 1024 * 1024;  // VoteRange::verify MAX_LEN (types.rs:448)

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

// Lane per block. Block i = buf[off[i] .. off[i] + len[i]); P || sig (then 8 zero bytes) is
// written at stage + round_up(off[i], 8), which stays inside the block's own span because
// the bincode is at least |P| + 128 bytes long. Writes happen only after the bytes they
// come from were read, so a malformed block never writes outside its span either.
__global__ void __launch_bounds__(256) k_block_parse(
    const uint8_t* __restrict__ buf, const uint64_t* __restrict__ off, const uint64_t* __restrict__ len, uint32_t n,
    const uint64_t* __restrict__ stakes, uint32_t n_auth, uint64_t epoch, uint64_t quorum_thr,
    uint8_t* __restrict__ stage, uint64_t* __restrict__ pre_off, uint64_t* __restrict__ pre_len,
    uint8_t* __restrict__ sig_out, uint32_t* __restrict__ key_idx, uint32_t* __restrict__ facts,
    uint8_t* __restrict__ claimed) {
  __shared__ uint32_t seen[16][256];  // per-lane authority bitmap (<= 512 authorities), [word][lane]
  const uint32_t t = threadIdx.x;
  const uint32_t i = blockIdx.x * 256 + t;
#pragma unroll
  for (int k = 0; k < 16; k++) seen[k][t] = 0;
  if (i >= n) return;
  const uint64_t o = off[i];
  const uint64_t so = (o + 7) & ~7ull;
  BcReader r{buf + o, len[i], 0, true};
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
      const uint32_t s = seen[wd][t];
      if (!(s & bit)) {
        seen[wd][t] = s | bit;
        stake += stakes[a];
      }
      quorum = stake > quorum_thr;
    }
  }
  // statements
  const uint64_t n_st = r.u64();
  bool vr_bad = false;
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
      if (s1 < s0 || s1 - s0 >= VR_MAX_LEN || s1 >= VR_MAX_LEN) vr_bad = true;
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
    pre_len[i] = plen;
    f = BF_PARSED | (ep == epoch ? BF_EPOCH_OK : 0u) | (me_a < n_auth ? BF_AUTHOR_OK : 0u) |
        (me_r == 0 ? BF_GENESIS : 0u) | (vr_bad ? BF_VR_BAD : 0u) | (quorum ? BF_QUORUM : 0u) |
        (inc_err << BF_INC_SHIFT);
    const uint64_t d0 = peek8(me_d), d1 = peek8(me_d + 8), d2 = peek8(me_d + 16), d3 = peek8(me_d + 24);
    uint4* cd = reinterpret_cast<uint4*>(claimed + 32 * (size_t)i);
    cd[0] = make_uint4((uint32_t)d0, (uint32_t)(d0 >> 32), (uint32_t)d1, (uint32_t)(d1 >> 32));
    cd[1] = make_uint4((uint32_t)d2, (uint32_t)(d2 >> 32), (uint32_t)d3, (uint32_t)(d3 >> 32));
  } else {
    pre_len[i] = 0;
#pragma unroll
    for (int q = 0; q < 16; q++) sw[q] = 0;
  }
  pre_off[i] = so;
  // a block rejected ahead of the signature check gets s = 2^256 - 1 (>= l): its verdict
  // does not depend on the signature, and s >= l keeps it out of the batch equation
  const bool sig_decides = parsed && (f & BF_EPOCH_OK) && (f & BF_AUTHOR_OK) && !(f & BF_GENESIS);
  if (!sig_decides) {
#pragma unroll
    for (int q = 8; q < 16; q++) sw[q] = 0xffffffffu;
  }
  uint4* so4 = reinterpret_cast<uint4*>(sig_out + 64 * (size_t)i);
#pragma unroll
  for (int q = 0; q < 4; q++) so4[q] = make_uint4(sw[4 * q], sw[4 * q + 1], sw[4 * q + 2], sw[4 * q + 3]);
  key_idx[i] = (parsed && me_a < n_auth) ? static_cast<uint32_t>(me_a) : 0u;
  facts[i] = f;
}

// status[i] in the order of StatementBlock::verify (types.rs:315-376)
__global__ void __launch_bounds__(256) k_block_verdict(const uint32_t* __restrict__ facts,
                                                       const uint8_t* __restrict__ claimed,
                                                       const uint8_t* __restrict__ digest,
                                                       const uint8_t* __restrict__ sig_status, uint32_t n,
                                                       uint8_t* __restrict__ status) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t f = facts[i];
  uint8_t st;
  if (!(f & BF_PARSED)) {
    st = MV_BLOCK_PARSE_ERROR;
  } else {
    const uint4* a = reinterpret_cast<const uint4*>(claimed + 32 * (size_t)i);
    const uint4* b = reinterpret_cast<const uint4*>(digest + 32 * (size_t)i);
    const uint4 a0 = a[0], a1 = a[1], b0 = b[0], b1 = b[1];
    const bool same = ((a0.x ^ b0.x) | (a0.y ^ b0.y) | (a0.z ^ b0.z) | (a0.w ^ b0.w) | (a1.x ^ b1.x) |
                       (a1.y ^ b1.y) | (a1.z ^ b1.z) | (a1.w ^ b1.w)) == 0;
    const uint32_t inc = (f >> BF_INC_SHIFT) & 0xffu;
    st = !same                      ? MV_BLOCK_DIGEST_MISMATCH
         : !(f & BF_EPOCH_OK)       ? MV_BLOCK_EPOCH_MISMATCH
         : !(f & BF_AUTHOR_OK)      ? MV_BLOCK_UNKNOWN_AUTHOR
         : (f & BF_GENESIS)         ? MV_BLOCK_GENESIS
         : sig_status[i] != MV_SIG_OK ? MV_BLOCK_SIG_INVALID
         : inc                      ? (uint8_t)inc
         : (f & BF_VR_BAD)          ? MV_BLOCK_VOTE_RANGE
         : !(f & BF_QUORUM)         ? MV_BLOCK_THRESHOLD_CLOCK
                                    : MV_BLOCK_OK;
  }
  status[i] = st;
}

}  // namespace mv

// ---------------------------------------------------------------- launchers
namespace mvk {

hipError_t launch_block_parse(const uint8_t* buf, const uint64_t* off, const uint64_t* len, uint32_t n,
                              const uint64_t* stakes, uint32_t n_auth, uint64_t epoch, uint64_t quorum_thr,
                              uint8_t* stage, uint64_t* pre_off, uint64_t* pre_len, uint8_t* sig, uint32_t* key_idx,
                              uint32_t* facts, uint8_t* claimed, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(mv::k_block_parse, dim3((n + 255) / 256), dim3(256), 0, s, buf, off, len, n, stakes, n_auth,
                     epoch, quorum_thr, stage, pre_off, pre_len, sig, key_idx, facts, claimed);
  return hipGetLastError();
}

hipError_t launch_block_verdict(const uint32_t* facts, const uint8_t* claimed, const uint8_t* digest,
                                const uint8_t* sig_status, uint32_t n, uint8_t* status, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(mv::k_block_verdict, dim3((n + 255) / 256), dim3(256), 0, s, facts, claimed, digest, sig_status,
                     n, status);
  return hipGetLastError();
}

}  // namespace mvk
