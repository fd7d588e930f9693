/* ORACLE / TEST INFRASTRUCTURE ONLY — see oracle.h.
 *
 * StatementBlock bincode parsing, digest pre-image and StatementBlock::verify.
 *   bincode layout   : field order of types.rs:93-114 (StatementBlock), types.rs:49-54
 *                      (BlockReference), types.rs:57-64 (BaseStatement), types.rs:31-35
 *                      (Vote), types.rs:384-394 (locators); SignatureBytes/BlockDigest
 *                      serialize as bytes with an exact-length check (crypto.rs:298-347).
 *                      bincode 1.3.3 `bincode::deserialize` defaults: little-endian,
 *                      fixint, u64 lengths, u32 enum tags, u8 Option/bool tags,
 *                      trailing bytes allowed.
 *   pre-image        : crypto.rs:85-128 (+ CryptoHash impls crypto.rs:150-170,
 *                      types.rs:661-691, Transaction AsBytes types.rs:751-755).
 *   verify order     : types.rs:315-376; VoteRange::verify types.rs:440-460;
 *                      threshold_clock_valid_non_genesis threshold_clock.rs:12-35;
 *                      quorum = stake > 2*total/3 (committee.rs:56-57,125-127).
 */
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "oracle.h"

typedef struct {
  const uint8_t* p;
  size_t n, pos;
  int err;
} cur_t;

static int take(cur_t* c, size_t k, const uint8_t** out) {
  if (c->err || k > c->n - c->pos) {
    c->err = 1;
    return 0;
  }
  *out = c->p + c->pos;
  c->pos += k;
  return 1;
}
static uint64_t rd_u64(cur_t* c) {
  const uint8_t* b;
  if (!take(c, 8, &b)) return 0;
  uint64_t v = 0;
  for (int i = 7; i >= 0; i--) v = (v << 8) | b[i];
  return v;
}
static uint32_t rd_u32(cur_t* c) {
  const uint8_t* b;
  if (!take(c, 4, &b)) return 0;
  return (uint32_t)b[0] | ((uint32_t)b[1] << 8) | ((uint32_t)b[2] << 16) | ((uint32_t)b[3] << 24);
}
static uint8_t rd_u8(cur_t* c) {
  const uint8_t* b;
  if (!take(c, 1, &b)) return 0;
  return b[0];
}
/* serialize_bytes of a fixed-size array: u64 length that must equal n */
static const uint8_t* rd_fixed_bytes(cur_t* c, size_t n) {
  uint64_t len = rd_u64(c);
  if (c->err) return NULL;
  if (len != n) {
    c->err = 1;
    return NULL;
  }
  const uint8_t* b;
  if (!take(c, n, &b)) return NULL;
  return b;
}

typedef struct {
  uint8_t* out;
  size_t cap, len;
} sink_t;
static void put(sink_t* s, const uint8_t* b, size_t k) {
  if (s->out && s->len + k <= s->cap) memcpy(s->out + s->len, b, k);
  s->len += k;
}
static void put_be64(sink_t* s, uint64_t v) {
  uint8_t b[8];
  for (int i = 0; i < 8; i++) b[i] = (uint8_t)(v >> (56 - 8 * i));
  put(s, b, 8);
}
static void put_byte(sink_t* s, uint8_t v) { put(s, &v, 1); }

typedef struct {
  uint64_t authority, round;
  const uint8_t* digest;
} ref_t;

static ref_t rd_ref(cur_t* c) {
  ref_t r;
  r.authority = rd_u64(c);
  r.round = rd_u64(c);
  r.digest = rd_fixed_bytes(c, 32);
  return r;
}
static void put_ref(sink_t* s, const ref_t* r) {
  put_be64(s, r->authority);
  put_be64(s, r->round);
  if (r->digest) put(s, r->digest, 32);
}

typedef struct {
  ref_t reference;
  uint64_t n_includes;
  size_t includes_pos; /* offset of the first include in the bincode bytes */
  uint64_t n_statements;
  size_t statements_pos;
  uint8_t time_be[16];
  uint8_t epoch_marker;
  uint64_t epoch;
  const uint8_t* signature;
} parsed_t;

/* Walks a statement; writes its pre-image bytes into s (may be a NULL sink).
 * *vr_bad set to the ORC_BLOCK_VOTE_RANGE* code of the first VoteRange that fails VoteRange::verify. */
static void walk_statement(cur_t* c, sink_t* s, int* vr_bad) {
  uint32_t tag = rd_u32(c);
  if (c->err) return;
  if (tag == 0) { /* Share(Transaction{data: Vec<u8>}) */
    uint64_t len = rd_u64(c);
    const uint8_t* b;
    if (!take(c, len, &b)) return;
    put_byte(s, 0);
    put(s, b, len); /* no length prefix in the pre-image */
  } else if (tag == 1) { /* Vote(TransactionLocator, Vote) */
    ref_t blk = rd_ref(c);
    uint64_t off = rd_u64(c);
    uint32_t vt = rd_u32(c);
    if (c->err) return;
    if (vt == 0) {
      put_byte(s, 1);
      put_ref(s, &blk);
      put_be64(s, off);
    } else if (vt == 1) {
      uint8_t opt = rd_u8(c);
      if (c->err) return;
      if (opt == 0) {
        put_byte(s, 2);
        put_ref(s, &blk);
        put_be64(s, off);
      } else if (opt == 1) {
        ref_t blk2 = rd_ref(c);
        uint64_t off2 = rd_u64(c);
        if (c->err) return;
        put_byte(s, 3);
        put_ref(s, &blk);
        put_be64(s, off);
        put_ref(s, &blk2);
        put_be64(s, off2);
      } else {
        c->err = 1;
      }
    } else {
      c->err = 1;
    }
  } else if (tag == 2) { /* VoteRange(TransactionLocatorRange) */
    ref_t blk = rd_ref(c);
    uint64_t start = rd_u64(c);
    uint64_t end = rd_u64(c);
    if (c->err) return;
    put_byte(s, 4);
    put_ref(s, &blk);
    put_be64(s, start);
    put_be64(s, end);
    const uint64_t MAX_LEN = 1024 * 1024;
    if (vr_bad && !*vr_bad) { /* VoteRange::verify (types.rs:440-460), checks in order */
      *vr_bad = end < start ? ORC_BLOCK_VOTE_RANGE
                : (end - start) >= MAX_LEN ? ORC_BLOCK_VOTE_RANGE_TOO_LONG
                : end >= MAX_LEN ? ORC_BLOCK_VOTE_RANGE_END_TOO_LARGE : 0;
    }
  } else {
    c->err = 1;
  }
}

/* Parse; returns 0 on success. Pre-image written to s when non-NULL. */
static int parse_block(const uint8_t* buf, size_t len, parsed_t* b, sink_t* s, int* vr_bad) {
  cur_t c = {buf, len, 0, 0};
  sink_t null_sink = {NULL, 0, 0};
  if (!s) s = &null_sink;
  b->reference = rd_ref(&c);
  b->n_includes = rd_u64(&c);
  if (c.err) return -1;
  put_be64(s, b->reference.authority);
  put_be64(s, b->reference.round);
  b->includes_pos = c.pos;
  for (uint64_t i = 0; i < b->n_includes && !c.err; i++) {
    ref_t r = rd_ref(&c);
    if (!c.err) put_ref(s, &r);
  }
  b->n_statements = rd_u64(&c);
  b->statements_pos = c.pos;
  for (uint64_t i = 0; i < b->n_statements && !c.err; i++) walk_statement(&c, s, vr_bad);
  const uint8_t* t;
  if (!take(&c, 16, &t)) return -1;
  for (int i = 0; i < 16; i++) b->time_be[i] = t[15 - i]; /* u128 LE -> BE */
  b->epoch_marker = rd_u8(&c);
  if (!c.err && b->epoch_marker > 1) c.err = 1; /* bincode bool */
  b->epoch = rd_u64(&c);
  b->signature = rd_fixed_bytes(&c, 64);
  if (c.err) return -1;
  put(s, b->time_be, 16);
  put_byte(s, b->epoch_marker);
  put_be64(s, b->epoch);
  return 0;
}

long orc_block_preimage(const uint8_t* bincode, size_t len, uint8_t* out, size_t cap) {
  parsed_t b;
  sink_t s = {out, cap, 0};
  if (parse_block(bincode, len, &b, &s, NULL) != 0) return -1;
  return (long)s.len;
}

/* `vks` (may be NULL): the committee's keys decoded once (orc_committee); else each verify
 * decodes its key from committee_pks */
static int block_verify(const uint8_t* bincode, size_t len, const uint8_t* committee_pks, const uint8_t* vks,
                        const uint64_t* stakes, uint32_t n_auth, uint64_t epoch, uint8_t msg_digest[32],
                        uint8_t block_digest[32]) {
  parsed_t b;
  int vr_bad = 0;
  long plen = orc_block_preimage(bincode, len, NULL, 0);
  if (plen < 0) return ORC_BLOCK_PARSE_ERROR;
  uint8_t* pre = (uint8_t*)malloc((size_t)plen + 64);
  sink_t s = {pre, (size_t)plen, 0};
  parse_block(bincode, len, &b, &s, &vr_bad);
  uint8_t msg[32], dig[32];
  orc_blake2b256(pre, (size_t)plen, msg); /* signed message, crypto.rs:174-187 */
  memcpy(pre + plen, b.signature, 64);
  orc_blake2b256(pre, (size_t)plen + 64, dig); /* block digest, crypto.rs:38-61 */
  free(pre);
  if (msg_digest) memcpy(msg_digest, msg, 32);
  if (block_digest) memcpy(block_digest, dig, 32);

  if (memcmp(dig, b.reference.digest, 32) != 0) return ORC_BLOCK_DIGEST_MISMATCH;
  if (b.epoch != epoch) return ORC_BLOCK_EPOCH_MISMATCH;
  if (b.reference.authority >= n_auth) return ORC_BLOCK_UNKNOWN_AUTHOR;
  if (b.reference.round == 0) return ORC_BLOCK_GENESIS;
  const int sig_st = vks ? orc_ed25519_verify_vk((const orc_vk*)(vks + orc_vk_size() * b.reference.authority),
                                                 b.signature, msg, 32)
                         : orc_ed25519_verify(committee_pks + 32 * b.reference.authority, b.signature, msg, 32);
  if (sig_st != ORC_SIG_OK) return ORC_BLOCK_SIG_INVALID;
  /* includes (types.rs:349-362), checked in order */
  cur_t c = {bincode, len, b.includes_pos, 0};
  uint64_t total = 0;
  for (uint32_t a = 0; a < n_auth; a++) total += stakes[a];
  uint64_t quorum_threshold = 2 * total / 3;
  for (uint64_t i = 0; i < b.n_includes; i++) {
    ref_t r = rd_ref(&c);
    if (r.authority >= n_auth) return ORC_BLOCK_INCLUDE_UNKNOWN_AUTHORITY;
    if (r.round >= b.reference.round) return ORC_BLOCK_INCLUDE_ROUND;
  }
  if (vr_bad) return vr_bad;
  /* threshold clock (threshold_clock.rs:12-35) */
  c.pos = b.includes_pos;
  c.err = 0;
  uint8_t seen[512];
  memset(seen, 0, sizeof seen);
  uint64_t stake = 0;
  int is_quorum = 0;
  for (uint64_t i = 0; i < b.n_includes; i++) {
    ref_t r = rd_ref(&c);
    if (r.round == b.reference.round - 1) {
      if (!seen[r.authority]) {
        seen[r.authority] = 1;
        stake += stakes[r.authority];
      }
      is_quorum = stake > quorum_threshold;
    }
  }
  if (!is_quorum) return ORC_BLOCK_THRESHOLD_CLOCK;
  return ORC_BLOCK_OK;
}

int orc_block_verify(const uint8_t* bincode, size_t len, const uint8_t* committee_pks, const uint64_t* stakes,
                     uint32_t n_auth, uint64_t epoch, uint8_t msg_digest[32], uint8_t block_digest[32]) {
  return block_verify(bincode, len, committee_pks, NULL, stakes, n_auth, epoch, msg_digest, block_digest);
}

/* The committee as a node holds it: keys decoded once (Committee::new, committee.rs:83-87) */
struct orc_committee {
  uint32_t n;
  uint64_t epoch;
  uint8_t* pks;
  uint64_t* stakes;
  uint8_t* vks; /* n x orc_vk_size() */
};

orc_committee* orc_committee_new(const uint8_t* pks, const uint64_t* stakes, uint32_t n, uint64_t epoch) {
  orc_committee* c = (orc_committee*)calloc(1, sizeof *c);
  c->n = n;
  c->epoch = epoch;
  c->pks = (uint8_t*)malloc(32 * (size_t)n + 1);
  c->stakes = (uint64_t*)malloc(8 * (size_t)n + 8);
  c->vks = (uint8_t*)malloc(orc_vk_size() * (size_t)n + 1);
  memcpy(c->pks, pks, 32 * (size_t)n);
  memcpy(c->stakes, stakes, 8 * (size_t)n);
  for (uint32_t i = 0; i < n; i++) orc_vk_init((orc_vk*)(c->vks + orc_vk_size() * i), pks + 32 * (size_t)i);
  return c;
}

void orc_committee_free(orc_committee* c) {
  if (!c) return;
  free(c->pks);
  free(c->stakes);
  free(c->vks);
  free(c);
}

int orc_block_verify_c(const orc_committee* c, const uint8_t* bincode, size_t len, uint8_t msg_digest[32],
                       uint8_t block_digest[32]) {
  return block_verify(bincode, len, c->pks, c->vks, c->stakes, c->n, c->epoch, msg_digest, block_digest);
}

typedef struct {
  const uint8_t* buf;
  const uint64_t *off, *len;
  const uint8_t* pks;
  const uint64_t* stakes;
  uint32_t n_auth;
  uint64_t epoch;
  uint8_t *status, *msgd, *blkd;
  const uint8_t* vks;
} bjob_t;

static void block_item(void* arg, size_t i) {
  bjob_t* j = (bjob_t*)arg;
  j->status[i] = (uint8_t)block_verify(j->buf + j->off[i], j->len[i], j->pks, j->vks, j->stakes, j->n_auth, j->epoch,
                                       j->msgd ? j->msgd + 32 * i : NULL, j->blkd ? j->blkd + 32 * i : NULL);
}

/* persistent pool (pool.c), one block per item */
void orc_block_verify_batch(const uint8_t* buf, const uint64_t* off, const uint64_t* len, size_t n,
                            const uint8_t* committee_pks, const uint64_t* stakes, uint32_t n_auth, uint64_t epoch,
                            uint8_t* status, uint8_t* msg_digests, uint8_t* block_digests, int threads) {
  bjob_t j = {buf, off, len, committee_pks, stakes, n_auth, epoch, status, msg_digests, block_digests, NULL};
  orc_parallel_for(n, threads, 1, block_item, &j);
}

void orc_block_verify_batch_c(const orc_committee* c, const uint8_t* buf, const uint64_t* off, const uint64_t* len,
                              size_t n, uint8_t* status, uint8_t* msg_digests, uint8_t* block_digests, int threads) {
  bjob_t j = {buf, off, len, c->pks, c->stakes, c->n, c->epoch, status, msg_digests, block_digests, c->vks};
  orc_parallel_for(n, threads, 1, block_item, &j);
}
