// k_block_walk: the whole block ingest and both BLAKE2b digests of a batch-size block call in
// ONE pass over the bincode, one lane per block.
//
// What it replaces: k_block_ingest (a wave per block: parse, checks, P || sig staged in HBM)
// followed by k_b2_lane (one lane per string over the staged pre-image). Per 2^20 config-4
// blocks that pair moved 29.3 GB (bincode 10.3 GB read, pre-image 8.8 GB written and 10.3 GB
// read back; profiles/r05/pmc/pmc_c4_*.txt); this kernel reads the 9.9 GB of bincode once.
//
// How: the lane walks its block's bincode front to back (bincode 1.3.3 defaults, data.rs:43-52;
// types.rs:93-114 StatementBlock) and emits the signed pre-image (crypto.rs:85-128 with the
// CryptoHash encodings of crypto.rs:150-170, types.rs:661-691, 751-755) piece by piece into its
// own LDS row (one piece per element, or per 64 bytes of a Share's payload, each read from one
// 80-byte window), hashing each 128-byte block as soon as it is complete. The checks of
// StatementBlock::verify that depend on the bincode (types.rs:333-362 includes, 440-460
// VoteRange, threshold_clock.rs:12-35) run on the same walk. The two digests share their
// common prefix as in k_b2_lane (Plan<true>), but the schedule is found on the way: the block
// in which P ends is compressed once as B2(P)'s final block (on a copy of the state) and then
// continued with the signature.
//
// Any failed read or check (a length past the block, a digest length other than 32, an
// unknown tag, vote or option, an epoch marker > 1, a signature length other than 64) makes
// the block a parse error, as ingest_lane's BcReader does: which check fails first never
// matters, because every failure gives the same verdict (MV_BLOCK_PARSE_ERROR, digests zeroed
// by k_block_verdict). tests/test_gpu_ingest.py runs every ingest case through this kernel
// (the batch_walk form) against the host codec and the oracle.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/mysti_verify.h"
#include "blake2b_quad.h"
#include "block_verdict.h"
#include "kernels.h"

namespace mv {
namespace bw {

using b2q::add64;
using b2q::IV;
using b2q::ror16;
using b2q::ror24;
using b2q::ror32;
using b2q::ror63;
using b2q::SIGMA;

#ifndef MV_WALK_ROW
#define MV_WALK_ROW 200  // (A/B builds may pad it to trade occupancy for L2 footprint)
#endif
constexpr uint32_t ROW = MV_WALK_ROW;  // bytes per lane: one message block + the longest piece (72 B)
static_assert(ROW >= 200 && ROW % 8 == 0, "a row holds a block and the longest piece");
constexpr uint64_t VR_MAX = 1024 * 1024;  // VoteRange::verify MAX_LEN (types.rs:448)

MV_DEV uint64_t ld64(const uint8_t* p) {
  uint64_t v;
  __builtin_memcpy(&v, p, 8);
  return v;
}
MV_DEV void st64(uint8_t* q, uint64_t v) { __builtin_memcpy(q, &v, 8); }
MV_DEV void st_be(uint8_t* q, uint64_t v) { st64(q, __builtin_bswap64(v)); }

enum : uint32_t { HDR, INC, NST, STMT, META, SIG, DONE };
constexpr uint32_t SUB_NONE = 0, SUB_SHARE = 1, SUB_REJ2 = 2;

struct CommitteeArgs {
  const uint64_t* stakes;
  uint32_t n_auth;
  uint64_t epoch, quorum_thr;
};
struct BlockOut {
  uint8_t* sig;
  uint32_t* key_idx;
  uint32_t* facts;
  uint8_t* claimed;
  uint8_t* md;
  uint8_t* bd;
};

// One block's walk: where it stands (phase, the element's bincode offset src, the phase's
// element count and index, a pending Share payload or Reject(Some) second locator), and the
// facts gathered so far. NW: words of the authority bitmap (32 authorities each).
template <int NW>
struct Walk {
  const uint8_t* blk;
  uint32_t len;  // bincode bytes of the block
  uint32_t phase, src, cnt, k, sub, rem, psrc;
  bool ok;
  uint64_t me_r;
  uint32_t me_a;  // the author, saturated to n_auth (only compared against it)
  uint32_t inc_code, vr_code;  // first failing include (code) and VoteRange (code), 0 = none
  uint64_t stake;
  uint32_t seen[NW];

  // a bound on the bytes left from bincode offset `at`
  MV_DEV bool fits(uint32_t at, uint32_t need) const { return at <= len && need <= len - at; }
};

// The bincode window a piece reads: WIN bytes from the element's offset, loaded before the piece
// is decoded (one round trip per piece, whichever branch its lanes take; the fields are then
// picked out of registers at compile-time offsets). Loads are clamped to start at most at the
// block's end, so they never leave the 16 readable bytes past it (mv_dev_verify_blocks).
constexpr int WIN = 80;  // the largest piece reads 76 bytes (a VoteRange)
struct Window {
  uint64_t x[WIN / 8];
};
MV_DEV void load_window(Window& wn, const uint8_t* blk, uint32_t at, uint32_t lim) {
#pragma unroll
  for (int j = 0; j < WIN / 16; j++) {
    uint64_t v[2];
    __builtin_memcpy(v, blk + min(at + 16u * j, lim), 16);  // one unaligned 16-byte load
    wn.x[2 * j] = v[0];
    wn.x[2 * j + 1] = v[1];
  }
}
// bytes [O, O + 8) of the window, little-endian
template <int O>
MV_DEV uint64_t wd(const Window& wn) {
  static_assert(O >= 0 && O + 8 <= WIN, "window field out of range");
  if constexpr (O % 8 == 0)
    return wn.x[O / 8];
  else
    return (wn.x[O / 8] >> (8 * (O % 8))) | (wn.x[O / 8 + 1] << (64 - 8 * (O % 8)));
}
template <int O>
MV_DEV uint32_t wd32(const Window& wn) {
  static_assert(O % 8 <= 4, "a 32-bit field inside one word");
  return (uint32_t)(wn.x[O / 8] >> (8 * (O % 8)));
}
template <int O>
MV_DEV uint32_t wb(const Window& wn) {
  return (uint32_t)(wn.x[O / 8] >> (8 * (O % 8))) & 0xffu;
}
// the 32 digest bytes of the BlockReference at window offset O (authority, round, u64 length,
// digest)
template <int O>
MV_DEV void st_dig(uint8_t* q, const Window& wn) {
  st64(q, wd<O + 24>(wn));
  st64(q + 8, wd<O + 32>(wn));
  st64(q + 16, wd<O + 40>(wn));
  st64(q + 24, wd<O + 48>(wn));
}

// Emits the next piece of the pre-image at q (<= 72 bytes; bytes past the returned length may
// be overwritten by the next piece) from the window wn of the element's bincode, and runs the
// checks of the element it belongs to; clears w.ok on the first failure. Returns the piece's
// length.
template <int NW>
MV_DEV uint32_t piece(Walk<NW>& w, uint8_t* q, const CommitteeArgs& ca, const Window& wn) {
  if (w.phase == HDR) {  // own reference (author, round, digest) and the include count
    if (!w.fits(0, 64)) {
      w.ok = false;
      return 0;
    }
    const uint64_t a = wd<0>(wn), r = wd<8>(wn), n_inc = wd<56>(wn);
    w.ok = wd<16>(wn) == 32 && n_inc <= (uint64_t)((w.len - 64) / 56);
    st_be(q, a);
    st_be(q + 8, r);
    w.me_a = a < ca.n_auth ? (uint32_t)a : ca.n_auth;
    w.me_r = r;
    w.cnt = (uint32_t)n_inc;
    w.src = 64;
    w.k = 0;
    w.phase = w.cnt ? INC : NST;
    return 16;
  }
  if (w.phase == INC) {  // includes (types.rs:349-362), threshold clock (threshold_clock.rs:12-35)
    const uint64_t a = wd<0>(wn), r = wd<8>(wn);
    w.ok = wd<16>(wn) == 32;
    st_be(q, a);
    st_be(q + 8, r);
    st_dig<0>(q + 16, wn);
    if (w.inc_code == 0)
      w.inc_code = a >= ca.n_auth ? (uint32_t)MV_BLOCK_INCLUDE_UNKNOWN_AUTHORITY
                                  : (r >= w.me_r ? (uint32_t)MV_BLOCK_INCLUDE_ROUND : 0u);
    if (w.me_r > 0 && r == w.me_r - 1 && a < ca.n_auth) {
      const uint32_t wdx = (uint32_t)a >> 5, bit = 1u << (a & 31);
      uint32_t s = 0;
#pragma unroll
      for (int j = 0; j < NW; j++) s |= wdx == (uint32_t)j ? w.seen[j] : 0u;
      if (!(s & bit)) {
#pragma unroll
        for (int j = 0; j < NW; j++) w.seen[j] |= wdx == (uint32_t)j ? bit : 0u;
        w.stake += ca.stakes[a];
      }
    }
    w.src += 56;
    if (++w.k == w.cnt) w.phase = NST;
    return 48;
  }
  if (w.phase == NST) {  // statement count (each statement takes >= 12 bincode bytes)
    if (!w.fits(w.src, 8)) {
      w.ok = false;
      return 0;
    }
    const uint64_t n_st = wd<0>(wn);
    w.src += 8;
    w.ok = n_st <= (uint64_t)((w.len - w.src) / 12);
    w.cnt = (uint32_t)n_st;
    w.k = 0;
    w.sub = SUB_NONE;
    w.phase = w.cnt ? STMT : META;
    return 0;
  }
  if (w.phase == STMT) {
    uint32_t n = 0;
    bool done = true;
    if (w.sub == SUB_SHARE) {  // Share payload, 64 bytes at a time (checked at its header; the
                               // words past the payload are junk the next piece overwrites)
#pragma unroll
      for (int j = 0; j < 8; j++)
        if (8u * j < w.rem) st64(q + 8 * j, wn.x[j]);
      n = min(w.rem, 64u);
      w.rem -= n;
      w.psrc += n;
      done = w.rem == 0;
    } else if (w.sub == SUB_REJ2) {  // Reject(Some): the second locator (its bytes were bounded
                                     // with the first; its digest length is checked here)
      w.ok = wd<16>(wn) == 32;
      st_be(q, wd<0>(wn));
      st_be(q + 8, wd<8>(wn));
      st_dig<0>(q + 16, wn);
      st_be(q + 48, wd<56>(wn));
      n = 56;
    } else {
      const uint32_t tag = w.fits(w.src, 4) ? wd32<0>(wn) : 3u;
      if (tag == 0) {  // Share(Transaction): u32 tag, u64 length, bytes -> 0, bytes
        if (!w.fits(w.src, 12) || wd<4>(wn) > (uint64_t)(w.len - w.src - 12)) {
          w.ok = false;
          return 0;
        }
        const uint32_t l = (uint32_t)wd<4>(wn);
        q[0] = 0;
        w.psrc = w.src + 12;
        w.rem = l;
        w.src += 12 + l;
        n = 1;
        done = l == 0;
        w.sub = SUB_SHARE;
      } else if (tag == 1) {  // Vote(locator, Accept | Reject(None) | Reject(Some(locator)))
        if (!w.fits(w.src, 72)) {
          w.ok = false;
          return 0;
        }
        const uint32_t vote = wd32<68>(wn);
        const uint32_t some = vote == 1 && w.fits(w.src, 73) ? wb<72>(wn) : 2u;
        const bool two = vote == 1 && some == 1;
        w.ok = wd<20>(wn) == 32 && (vote == 0 || some <= 1) && (!two || w.fits(w.src, 137));
        q[0] = (uint8_t)(vote == 0 ? 1 : (two ? 3 : 2));
        st_be(q + 1, wd<4>(wn));
        st_be(q + 9, wd<12>(wn));
        st_dig<4>(q + 17, wn);
        st_be(q + 49, wd<60>(wn));
        n = 57;
        if (two) {
          w.psrc = w.src + 73;
          w.sub = SUB_REJ2;
          done = false;
        }
        w.src += vote == 0 ? 72 : (two ? 137 : 73);
      } else if (tag == 2) {  // VoteRange(locator range): VoteRange::verify (types.rs:440-460)
        if (!w.fits(w.src, 76)) {
          w.ok = false;
          return 0;
        }
        const uint64_t s0 = wd<60>(wn), s1 = wd<68>(wn);
        w.ok = wd<20>(wn) == 32;
        q[0] = 4;
        st_be(q + 1, wd<4>(wn));
        st_be(q + 9, wd<12>(wn));
        st_dig<4>(q + 17, wn);
        st_be(q + 49, s0);
        st_be(q + 57, s1);
        if (w.vr_code == 0) w.vr_code = s1 < s0 ? 1u : (s1 - s0 >= VR_MAX ? 2u : (s1 >= VR_MAX ? 3u : 0u));
        w.src += 76;
        n = 65;
      } else {
        w.ok = false;
        return 0;
      }
    }
    if (done) {
      w.sub = SUB_NONE;
      if (++w.k == w.cnt) w.phase = META;
    }
    return n;
  }
  // META: creation time (u128 -> big-endian high, low), epoch marker, epoch; then u64 64 and the
  // signature (97 bincode bytes in all)
  if (!w.fits(w.src, 97)) {
    w.ok = false;
    return 0;
  }
  const uint32_t marker = wb<16>(wn);
  w.ok = marker <= 1 && wd<25>(wn) == 64;
  st_be(q, wd<8>(wn));
  st_be(q + 8, wd<0>(wn));
  q[16] = (uint8_t)marker;
  st_be(q + 17, wd<17>(wn));
  w.phase = SIG;
  return 25;
}

// MV_LG: BLAKE2b's G on four state words and two message words (RFC 7693 §3.1)
#define MV_LG(a, bb, c, d, x, y) \
  a = add64(add64(a, bb), x);    \
  d = ror32(d ^ a);              \
  c = add64(c, d);               \
  bb = ror24(bb ^ c);            \
  a = add64(add64(a, bb), y);    \
  d = ror16(d ^ a);              \
  c = add64(c, d);               \
  bb = ror63(bb ^ c);

// Blocks [0, n) of buf at off[i] (len[i] bytes), 64 per 64-lane workgroup.
template <int NW>
__global__ void __launch_bounds__(64) k_block_walk(const uint8_t* __restrict__ buf, const uint64_t* __restrict__ off,
                                                   const uint64_t* __restrict__ len, uint32_t n, CommitteeArgs ca,
                                                   BlockOut out) {
  __shared__ uint64_t rows[64 * ROW / 8];
  const uint32_t lane = threadIdx.x;
  const uint32_t i = blockIdx.x * 64 + lane;
  uint8_t* const row = reinterpret_cast<uint8_t*>(rows) + ROW * lane;
  uint64_t* const row64 = rows + (ROW / 8) * lane;
  Walk<NW> w;
  w.blk = buf + (i < n ? off[i] : 0);
  const uint64_t L64 = i < n ? len[i] : 0;
  w.len = L64 > 0xffffffffull ? 0xffffffffu : (uint32_t)L64;
  const uint32_t lim = min(w.len, 0xffffff00u);  // window loads start at most here (the block's end)
  w.phase = HDR;
  w.src = w.cnt = w.k = w.rem = w.psrc = 0;
  w.sub = SUB_NONE;
  w.ok = i < n && L64 <= 0xffffffffull;
  w.me_r = 0;
  w.me_a = 0;
  w.inc_code = w.vr_code = 0;
  w.stake = 0;
#pragma unroll
  for (int j = 0; j < NW; j++) w.seen[j] = 0;
  bool live = w.ok, pdone = false;
  uint32_t pos = 0, plen = 0;
  uint64_t blocks = 0;  // message blocks of P || sig compressed so far
  uint64_t h[8];
#pragma unroll
  for (int k = 0; k < 8; k++) h[k] = IV[k];
  h[0] ^= 0x01010020ull;  // depth 1, fanout 1, nn = 32
  while (__ballot(live)) {
    // fill the row up to a whole block, P's end (its final block goes first), or the end
    while (live && w.ok && pos < 128 && w.phase != DONE) {
      if (w.phase == SIG) {
        if (!pdone) break;
        const uint8_t* e = w.blk + w.src + 33;
#pragma unroll
        for (int j = 0; j < 8; j++) st64(row + pos + 8 * j, ld64(e + 8 * j));
        w.phase = DONE;
        pos += 64;
      } else {
        Window wn;
        load_window(wn, w.blk, w.phase == STMT && w.sub != SUB_NONE ? w.psrc : w.src, lim);
        pos += piece(w, row + pos, ca, wn);
        if (w.phase == SIG && w.ok) plen = (uint32_t)(128 * blocks) + pos;  // P ends here
      }
    }
    if (live && !w.ok) live = false;  // a parse error: no digests (the verdict zeroes them)
    // this step's compression: P's final block (mfin, on a copy of the state), the last block
    // of P || sig (fin), or a full block in between
    const bool mfin = live && w.phase == SIG && !pdone && pos <= 128;
    const bool fin = live && !mfin && w.phase == DONE && pos <= 128;
    const uint32_t lrel = mfin || fin ? pos : 128u;
    const uint64_t t = mfin ? (uint64_t)plen : (fin ? (uint64_t)plen + 64 : 128 * (blocks + 1));
    uint64_t m[16];
#pragma unroll
    for (int j = 0; j < 16; j++) {
      uint64_t v = row64[j];
      const uint32_t at = 8 * j;
      if (at + 8 > lrel) v = at >= lrel ? 0ull : v & ((1ull << (8 * (lrel - at))) - 1);
      m[j] = v;
    }
    uint64_t v[16];
#pragma unroll
    for (int k = 0; k < 8; k++) {
      v[k] = h[k];
      v[8 + k] = IV[k];
    }
    v[12] ^= t;
    v[14] = mfin || fin ? ~v[14] : v[14];
#pragma unroll
    for (int r = 0; r < 12; r++) {
      MV_LG(v[0], v[4], v[8], v[12], m[SIGMA[r][0]], m[SIGMA[r][1]])
      MV_LG(v[1], v[5], v[9], v[13], m[SIGMA[r][2]], m[SIGMA[r][3]])
      MV_LG(v[2], v[6], v[10], v[14], m[SIGMA[r][4]], m[SIGMA[r][5]])
      MV_LG(v[3], v[7], v[11], v[15], m[SIGMA[r][6]], m[SIGMA[r][7]])
      MV_LG(v[0], v[5], v[10], v[15], m[SIGMA[r][8]], m[SIGMA[r][9]])
      MV_LG(v[1], v[6], v[11], v[12], m[SIGMA[r][10]], m[SIGMA[r][11]])
      MV_LG(v[2], v[7], v[8], v[13], m[SIGMA[r][12]], m[SIGMA[r][13]])
      MV_LG(v[3], v[4], v[9], v[14], m[SIGMA[r][14]], m[SIGMA[r][15]])
    }
    if (mfin) {  // B2(P) = msg
      uint64_t* o = reinterpret_cast<uint64_t*>(out.md + 32 * (size_t)i);
#pragma unroll
      for (int k = 0; k < 4; k++) o[k] = h[k] ^ v[k] ^ v[8 + k];
      pdone = true;
    } else if (fin) {  // B2(P || sig) = the block digest
      uint64_t* o = reinterpret_cast<uint64_t*>(out.bd + 32 * (size_t)i);
#pragma unroll
      for (int k = 0; k < 4; k++) o[k] = h[k] ^ v[k] ^ v[8 + k];
      live = false;
    } else if (live) {
#pragma unroll
      for (int k = 0; k < 8; k++) h[k] ^= v[k] ^ v[8 + k];
      blocks++;
      // the bytes emitted past the block move to the row's start
#pragma unroll
      for (int j = 0; j < 9; j++) row64[j] = row64[16 + j];
      pos -= 128;
    }
  }
  if (i >= n) return;
  // per-block outputs (ingest_lane's): facts, claimed digest, signature (s = 2^256 - 1 unless
  // the signature decides the verdict), key index
  const bool parsed = w.ok && w.phase == DONE;
  uint32_t f = 0;
  if (parsed)
    f = BF_PARSED | (ld64(w.blk + w.src + 17) == ca.epoch ? BF_EPOCH_OK : 0u) |
        (w.me_a < ca.n_auth ? BF_AUTHOR_OK : 0u) | (w.me_r == 0 ? BF_GENESIS : 0u) | (w.vr_code << BF_VR_SHIFT) |
        (w.stake > ca.quorum_thr ? BF_QUORUM : 0u) | (w.inc_code << BF_INC_SHIFT);
  const bool sig_decides = parsed && (f & BF_EPOCH_OK) && (f & BF_AUTHOR_OK) && !(f & BF_GENESIS);
  uint64_t sw[8];
#pragma unroll
  for (int q = 0; q < 8; q++) {
    sw[q] = parsed ? ld64(w.blk + w.src + 33 + 8 * q) : 0ull;
    if (q >= 4 && !sig_decides) sw[q] = ~0ull;
  }
  uint4* so4 = reinterpret_cast<uint4*>(out.sig + 64 * (size_t)i);
#pragma unroll
  for (int q = 0; q < 4; q++)
    so4[q] = make_uint4((uint32_t)sw[2 * q], (uint32_t)(sw[2 * q] >> 32), (uint32_t)sw[2 * q + 1],
                        (uint32_t)(sw[2 * q + 1] >> 32));
  if (parsed) {
    uint4* cd = reinterpret_cast<uint4*>(out.claimed + 32 * (size_t)i);
    const uint64_t d0 = ld64(w.blk + 24), d1 = ld64(w.blk + 32), d2 = ld64(w.blk + 40), d3 = ld64(w.blk + 48);
    cd[0] = make_uint4((uint32_t)d0, (uint32_t)(d0 >> 32), (uint32_t)d1, (uint32_t)(d1 >> 32));
    cd[1] = make_uint4((uint32_t)d2, (uint32_t)(d2 >> 32), (uint32_t)d3, (uint32_t)(d3 >> 32));
  }
  out.key_idx[i] = parsed && w.me_a < ca.n_auth ? w.me_a : 0u;
  out.facts[i] = f;
}
#undef MV_LG

}  // namespace bw
}  // namespace mv

namespace mvk {

hipError_t launch_block_walk(const uint8_t* buf, const uint64_t* off, const uint64_t* len, uint32_t n,
                             const uint64_t* stakes, uint32_t n_auth, uint64_t epoch, uint64_t quorum_thr,
                             uint8_t* sig, uint32_t* key_idx, uint32_t* facts, uint8_t* claimed, uint8_t* md,
                             uint8_t* bd, hipStream_t s) {
  if (n == 0) return hipSuccess;
  if (n_auth > 512) return hipErrorInvalidValue;
  const mv::bw::CommitteeArgs ca{stakes, n_auth, epoch, quorum_thr};
  const mv::bw::BlockOut out{sig, key_idx, facts, claimed, md, bd};
  if (n_auth <= 128)  // config 4's committee: a 4-word authority bitmap in VGPRs
    hipLaunchKernelGGL(mv::bw::k_block_walk<4>, dim3((n + 63) / 64), dim3(64), 0, s, buf, off, len, n, ca, out);
  else
    hipLaunchKernelGGL(mv::bw::k_block_walk<16>, dim3((n + 63) / 64), dim3(64), 0, s, buf, off, len, n, ca, out);
  return hipGetLastError();
}

}  // namespace mvk
