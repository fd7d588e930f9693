/* ORACLE / TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference's StatementBlock crypto path, used by tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg as the CHECKER. The
 * product (mysticeti_amd/, libmysti_verify.so) never links or calls it.
 *
 * What it restates (reference @ /root/reference, hrubaanna/mysticeti 2025-02-04):
 *   - pre-image   : mysticeti-core/src/crypto.rs:85-128, crypto.rs:150-170,
 *                   types.rs:661-691, types.rs:751-755
 *   - digests     : crypto.rs:38-61 (block digest), crypto.rs:174-189 (signed msg)
 *   - verify order: types.rs:315-376, threshold_clock.rs:12-35, types.rs:440-460
 *   - bincode     : types.rs:49-114 field order, data.rs:43-52 (bincode 1.3.3
 *                   defaults: LE fixint, u64 lengths, u32 enum tags)
 *   - third-party crates (NOT vendored, restated from their published algorithms):
 *       blake2 0.10.6 Blake2b<U32>      -> RFC 7693, nn=32, kk=0
 *       sha2 0.9.9 Sha512                -> FIPS 180-4
 *       ed25519-consensus 2.1.0 verify   -> ZIP-215 (cofactored, non-canonical y ok)
 *       curve25519-dalek-ng 4.1.1        -> u64 backend structure: 5x51-bit limbs,
 *                                           Straus wNAF-5 (A) / wNAF-8 (B)
 * Parity pinning: tests/golden (hashlib, libsodium 1.0.18 RFC 8032 signing, the
 * pure-Python ZIP-215 predicate in oracle/zip215.py). Reference-side (Rust)
 * parity is unpinned: no cargo in this image, and the reference's own tests stub
 * crypto out (crypto.rs:63-75, 191-194, 225-237).
 */
#ifndef MV_ORACLE_H
#define MV_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- hashes ---- */
void orc_blake2b256(const uint8_t* in, size_t len, uint8_t out[32]);
void orc_sha512(const uint8_t* in, size_t len, uint8_t out[64]);

/* ---- ed25519 (ZIP-215) ---- */
enum { ORC_SIG_OK = 0, ORC_SIG_INVALID = 1, ORC_SIG_MALFORMED_KEY = 2 };
int orc_ed25519_verify(const uint8_t pk[32], const uint8_t sig[64], const uint8_t* msg, size_t msg_len);
void orc_ed25519_pubkey(const uint8_t seed[32], uint8_t pk[32]);
void orc_ed25519_sign(const uint8_t seed[32], const uint8_t* msg, size_t msg_len, uint8_t sig[64]);
/* A decoded verification key (bytes + -A), as ed25519_consensus::VerificationKey holds it. */
typedef struct orc_vk orc_vk;
size_t orc_vk_size(void);
int orc_vk_init(orc_vk* vk, const uint8_t pk[32]); /* 1 if pk decodes */
int orc_ed25519_verify_vk(const orc_vk* vk, const uint8_t sig[64], const uint8_t* msg, size_t msg_len);
/* ZIP-215 decode of a point encoding; returns 1 if it decodes. */
int orc_point_decodes(const uint8_t enc[32]);
/* x mod l for a 64-byte little-endian integer (Scalar::from_bytes_wide). */
void orc_scalar_reduce_wide(const uint8_t in[64], uint8_t out[32]);

/* batch verify on `threads` host threads (0 = all cores); msgs are 32 B each. */
/* pool.c: fn(ctx, i) for i in [0, n) on `threads` threads (the caller + persistent workers),
 * handed out `grain` items at a time. */
typedef void (*orc_item_fn)(void* ctx, size_t i);
void orc_parallel_for(size_t n, int threads, size_t grain, orc_item_fn fn, void* ctx);

void orc_ed25519_verify_batch(const uint8_t* pk, const uint8_t* sig, const uint8_t* msg32, size_t n,
                              uint8_t* status, int threads);
void orc_ed25519_sign_batch(const uint8_t* seed, const uint8_t* msg32, size_t n, uint8_t* pk, uint8_t* sig,
                            int threads);

/* ---- StatementBlock (bincode Data<StatementBlock> bytes) ---- */
/* Block verification statuses, in the error order of StatementBlock::verify
 * (types.rs:315-376). Mirrors include/mysti_verify.h MV_BLOCK_*. */
enum {
  ORC_BLOCK_OK = 0,
  ORC_BLOCK_PARSE_ERROR = 1,
  ORC_BLOCK_DIGEST_MISMATCH = 2,
  ORC_BLOCK_EPOCH_MISMATCH = 3,
  ORC_BLOCK_UNKNOWN_AUTHOR = 4,
  ORC_BLOCK_GENESIS = 5,
  ORC_BLOCK_SIG_INVALID = 6,
  ORC_BLOCK_INCLUDE_UNKNOWN_AUTHORITY = 7,
  ORC_BLOCK_INCLUDE_ROUND = 8,
  ORC_BLOCK_VOTE_RANGE = 9,             /* end < start */
  ORC_BLOCK_THRESHOLD_CLOCK = 10,
  ORC_BLOCK_VOTE_RANGE_TOO_LONG = 11,     /* end - start >= 2^20 */
  ORC_BLOCK_VOTE_RANGE_END_TOO_LARGE = 12, /* end >= 2^20 */
};

/* Parse bincode bytes and write the signed pre-image (crypto.rs:85-128).
 * Returns pre-image length, or -1 on a parse error. `out` may be NULL (length only). */
long orc_block_preimage(const uint8_t* bincode, size_t len, uint8_t* out, size_t cap);
/* Full StatementBlock::verify against a committee (pks[n][32], stakes[n], epoch).
 * msg_digest/block_digest (may be NULL) receive the two Blake2b-256 outputs. */
int orc_block_verify(const uint8_t* bincode, size_t len, const uint8_t* committee_pks, const uint64_t* stakes,
                     uint32_t n_auth, uint64_t epoch, uint8_t msg_digest[32], uint8_t block_digest[32]);
void orc_block_verify_batch(const uint8_t* buf, const uint64_t* off, const uint64_t* len, size_t n,
                            const uint8_t* committee_pks, const uint64_t* stakes, uint32_t n_auth, uint64_t epoch,
                            uint8_t* status, uint8_t* msg_digests, uint8_t* block_digests, int threads);
/* A committee with its keys decoded once, as the reference's Committee holds them (the CPU
 * baseline legs use it; orc_block_verify decodes the author's key on every call). */
typedef struct orc_committee orc_committee;
orc_committee* orc_committee_new(const uint8_t* pks, const uint64_t* stakes, uint32_t n, uint64_t epoch);
void orc_committee_free(orc_committee* c);
int orc_block_verify_c(const orc_committee* c, const uint8_t* bincode, size_t len, uint8_t msg_digest[32],
                       uint8_t block_digest[32]);
void orc_block_verify_batch_c(const orc_committee* c, const uint8_t* buf, const uint64_t* off, const uint64_t* len,
                              size_t n, uint8_t* status, uint8_t* msg_digests, uint8_t* block_digests, int threads);

/* ---- WAL replay check (wal.c) ---- */
enum { ORC_WAL_OK = 0, ORC_WAL_CRC_MISMATCH = 1, ORC_WAL_NONZERO_CRC_LEN0 = 2, ORC_WAL_BAD_LENGTH = 3 };
/* crc32fast::hash (CRC-32/ISO-HDLC): orc_crc32 folds with PCLMULQDQ where the CPU has it (as
 * crc32fast does on x86_64), orc_crc32_table is the byte-at-a-time table form */
uint32_t orc_crc32(const uint8_t* p, size_t n);
uint32_t orc_crc32_table(const uint8_t* p, size_t n);
void orc_crc32_batch(const uint8_t* buf, const uint64_t* off, const uint64_t* len, size_t n, uint32_t* out);
/* WalWriter::writev positions of n entries of payload_len bytes from writer position `start`;
 * returns the writer position after them. */
uint64_t orc_wal_layout(const uint64_t* payload_len, size_t n, uint32_t map_bits, uint64_t start, uint64_t* pos);
/* WalReader::iter_until over img[0, size) up to end_pos: entries (position, tag, payload length,
 * ORC_WAL_* status) in order, stopping after the first failing one; returns the entry count
 * (entries past cap are counted, not written). */
uint64_t orc_wal_iter(const uint8_t* img, uint64_t size, uint64_t end_pos, uint32_t map_bits, uint64_t* pos,
                      uint32_t* tag, uint32_t* len, uint8_t* status, uint64_t cap);

#ifdef __cplusplus
}
#endif
#endif
