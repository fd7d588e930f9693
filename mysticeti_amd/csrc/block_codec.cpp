// See block_codec.h for the reference citations.
#include "block_codec.h"

#include <string.h>

#include "../../include/mysti_verify.h"

namespace mvh {
namespace {

class Reader {
 public:
  Reader(const uint8_t* p, size_t n) : p_(p), n_(n) {}
  bool ok() const { return ok_; }
  size_t pos() const { return pos_; }
  const uint8_t* bytes(size_t k) {
    if (!ok_ || k > n_ - pos_) {
      ok_ = false;
      return nullptr;
    }
    const uint8_t* r = p_ + pos_;
    pos_ += k;
    return r;
  }
  uint64_t u64() {
    const uint8_t* b = bytes(8);
    uint64_t v = 0;
    if (b) memcpy(&v, b, 8);  // little-endian host (x86-64)
    return v;
  }
  uint32_t u32() {
    const uint8_t* b = bytes(4);
    uint32_t v = 0;
    if (b) memcpy(&v, b, 4);
    return v;
  }
  uint8_t u8() {
    const uint8_t* b = bytes(1);
    return b ? *b : 0;
  }
  // serialize_bytes of a [u8; N]: u64 length that must equal N
  const uint8_t* fixed(size_t n) {
    uint64_t l = u64();
    if (ok_ && l != n) ok_ = false;
    return bytes(n);
  }
  void fail() { ok_ = false; }

 private:
  const uint8_t* p_;
  size_t n_;
  size_t pos_ = 0;
  bool ok_ = true;
};

class Writer {
 public:
  Writer(uint8_t* p, size_t cap) : p_(p), cap_(cap) {}
  void raw(const uint8_t* b, size_t k) {
    if (p_ && len_ + k <= cap_) memcpy(p_ + len_, b, k);
    len_ += k;
  }
  void be64(uint64_t v) {
    uint8_t b[8];
    for (int i = 0; i < 8; i++) b[i] = (uint8_t)(v >> (56 - 8 * i));
    raw(b, 8);
  }
  void byte(uint8_t v) { raw(&v, 1); }
  size_t len() const { return len_; }

 private:
  uint8_t* p_;
  size_t cap_;
  size_t len_ = 0;
};

struct Ref {
  uint64_t authority = 0, round = 0;
  const uint8_t* digest = nullptr;
};

Ref read_ref(Reader& r) {
  Ref x;
  x.authority = r.u64();
  x.round = r.u64();
  x.digest = r.fixed(32);
  return x;
}
void write_ref(Writer& w, const Ref& x) {
  w.be64(x.authority);
  w.be64(x.round);
  if (x.digest) w.raw(x.digest, 32);
}

constexpr uint64_t kMaxRangeLen = 1024 * 1024;  // VoteRange::verify MAX_LEN (types.rs:448)

}  // namespace

bool parse_block(const uint8_t* buf, size_t len, const Committee* committee, uint8_t* pre, size_t cap,
                 BlockFacts& f) {
  Reader r(buf, len);
  Writer w(pre, cap);
  f = BlockFacts();
  Ref me = read_ref(r);
  if (!r.ok()) return false;
  f.author = me.authority;
  f.round = me.round;
  memcpy(f.claimed_digest, me.digest, 32);
  w.be64(me.authority);
  w.be64(me.round);

  // includes: digest pre-image, include checks (types.rs:349-362), threshold clock
  uint64_t n_inc = r.u64();
  if (!r.ok()) return false;
  const uint32_t n_auth = committee ? committee->size() : 0;
  uint64_t stake = 0;
  bool quorum = false;
  std::vector<uint8_t> seen(committee ? n_auth : 0, 0);
  for (uint64_t i = 0; i < n_inc; i++) {
    Ref inc = read_ref(r);
    if (!r.ok()) return false;
    write_ref(w, inc);
    if (!committee) continue;
    if (f.include_error == 0) {
      if (inc.authority >= n_auth)
        f.include_error = MV_BLOCK_INCLUDE_UNKNOWN_AUTHORITY;
      else if (inc.round >= me.round)
        f.include_error = MV_BLOCK_INCLUDE_ROUND;
    }
    if (me.round > 0 && inc.round == me.round - 1 && inc.authority < n_auth) {
      if (!seen[inc.authority]) {
        seen[inc.authority] = 1;
        stake += committee->stakes[inc.authority];
      }
      quorum = stake > committee->quorum_threshold;
    }
  }
  f.threshold_ok = quorum;

  uint64_t n_st = r.u64();
  if (!r.ok()) return false;
  for (uint64_t i = 0; i < n_st; i++) {
    uint32_t tag = r.u32();
    if (!r.ok()) return false;
    if (tag == 0) {  // Share(Transaction): raw bytes, no length in the pre-image
      uint64_t l = r.u64();
      const uint8_t* b = r.bytes(l);
      if (!r.ok()) return false;
      w.byte(0);
      w.raw(b, l);
    } else if (tag == 1) {  // Vote(TransactionLocator, Vote)
      Ref blk = read_ref(r);
      uint64_t off = r.u64();
      uint32_t vote = r.u32();
      if (!r.ok()) return false;
      if (vote == 0) {
        w.byte(1);
        write_ref(w, blk);
        w.be64(off);
      } else if (vote == 1) {
        uint8_t some = r.u8();
        if (!r.ok()) return false;
        if (some == 0) {
          w.byte(2);
          write_ref(w, blk);
          w.be64(off);
        } else if (some == 1) {
          Ref blk2 = read_ref(r);
          uint64_t off2 = r.u64();
          if (!r.ok()) return false;
          w.byte(3);
          write_ref(w, blk);
          w.be64(off);
          write_ref(w, blk2);
          w.be64(off2);
        } else {
          return false;
        }
      } else {
        return false;
      }
    } else if (tag == 2) {  // VoteRange(TransactionLocatorRange)
      Ref blk = read_ref(r);
      uint64_t start = r.u64(), end = r.u64();
      if (!r.ok()) return false;
      w.byte(4);
      write_ref(w, blk);
      w.be64(start);
      w.be64(end);
      // VoteRange::verify (types.rs:440-460): its three checks in order; the first failing range decides
      if (!f.vote_range_error)
        f.vote_range_error = end < start                    ? MV_BLOCK_VOTE_RANGE
                             : end - start >= kMaxRangeLen ? MV_BLOCK_VOTE_RANGE_TOO_LONG
                             : end >= kMaxRangeLen         ? MV_BLOCK_VOTE_RANGE_END_TOO_LARGE
                                                           : 0;
    } else {
      return false;
    }
  }
  const uint8_t* t = r.bytes(16);  // u128 LE
  uint8_t marker = r.u8();
  if (r.ok() && marker > 1) r.fail();  // bincode bool
  f.epoch = r.u64();
  const uint8_t* sig = r.fixed(64);
  if (!r.ok()) return false;
  uint8_t tbe[16];
  for (int i = 0; i < 16; i++) tbe[i] = t[15 - i];
  w.raw(tbe, 16);
  w.byte(marker);
  w.be64(f.epoch);
  memcpy(f.signature, sig, 64);
  f.preimage_len = w.len();
  f.parsed = true;
  return true;
}

uint8_t block_verdict(const BlockFacts& f, const Committee& c, const uint8_t computed_digest[32], uint8_t sig_status) {
  if (!f.parsed) return MV_BLOCK_PARSE_ERROR;
  if (memcmp(computed_digest, f.claimed_digest, 32) != 0) return MV_BLOCK_DIGEST_MISMATCH;
  if (f.epoch != c.epoch) return MV_BLOCK_EPOCH_MISMATCH;
  if (f.author >= c.size()) return MV_BLOCK_UNKNOWN_AUTHOR;
  if (f.round == 0) return MV_BLOCK_GENESIS;
  if (sig_status != MV_SIG_OK) return MV_BLOCK_SIG_INVALID;
  if (f.include_error) return f.include_error;
  if (f.vote_range_error) return f.vote_range_error;
  if (!f.threshold_ok) return MV_BLOCK_THRESHOLD_CLOCK;
  return MV_BLOCK_OK;
}

}  // namespace mvh
