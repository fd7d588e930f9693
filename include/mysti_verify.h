/* mysti_verify.h — C ABI of the MI355X StatementBlock verification engine.
 *
 * Drop-in boundary for the per-block crypto of hrubaanna/mysticeti
 * (reference @ 2025-02-04). Each entry point names the reference interface it
 * replaces (paths relative to the reference repo):
 *
 *   mv_blake2b256          BlockHasher = blake2::Blake2b<U32> (mysticeti-core/src/crypto.rs:34),
 *                          as used by BlockDigest::new (crypto.rs:38-61)
 *   mv_ed25519_verify      PublicKey::verify_block -> ed25519_consensus::VerificationKey::verify
 *                          (crypto.rs:174-189; ZIP-215 semantics of ed25519-consensus 2.1.0)
 *   mv_ed25519_sign        Signer::sign_block -> ed25519_consensus::SigningKey::sign
 *                          (crypto.rs:199-223; RFC 8032)
 *   mv_set_committee       Committee::get_public_key / stake (committee.rs:56-87); the
 *                          VerificationKey decode that happens once per authority
 *   mv_verify_blocks       the loop `for block in blocks { block.verify(&committee) }` of
 *                          NetworkSyncer::process_blocks (net_sync.rs:331-375) over
 *                          StatementBlock::verify (types.rs:315-376), on Data<StatementBlock>
 *                          bincode bytes (data.rs:43-52)
 *   mv_dev_ed25519_verify_batch
 *                          ed25519_consensus::batch::Verifier (the ZIP-215 batch rule, which agrees
 *                          with VerificationKey::verify) over a whole batch, with an exact
 *                          per-signature fallback: per-item verdicts equal mv_ed25519_verify's
 *   mv_dev_*               the same computations on device-resident buffers (HBM in, HBM out)
 *   mv_crc32               crc32fast::hash (crc32fast 1.3.2, Cargo.lock:777), as the WAL uses it
 *                          (mysticeti-core/src/wal.rs:173-177, :250)
 *   mv_wal_verify          WalReader::iter_until + WalIterator::next over WalReader::try_read
 *                          (wal.rs:226-346): the entry walk and crc check of the WAL replay in
 *                          BlockStore::open (block_store.rs:66)
 *   mv_wal_layout          WalWriter::writev position arithmetic (wal.rs:150-188), host only
 *   mv_frame_blocks        the block byte strings of received NetworkMessage frames
 *                          (Network::handle_read_stream, network.rs:400-447), host only
 *
 * Conventions
 *   - The caller owns every buffer passed in and out; they must stay valid for the call.
 *     The library copies host inputs into its own pinned staging and device memory.
 *   - Return value: MV_OK (0) or a negative MV_E_* code; mv_last_error() gives text.
 *     Per-item verdicts go to caller arrays: a rejected signature is not an error.
 *   - Host-buffer calls are synchronous and thread-safe on one context. mv_verify_blocks callers
 *     are coalesced (a submission queue merges concurrent calls into shared device passes);
 *     the other host-buffer calls take the context in turn.
 *   - A context spans the devices in mv_config.device_mask; host-buffer calls shard
 *     their items across them (no collective: each device returns its slice of verdicts).
 */
#ifndef MYSTI_VERIFY_H
#define MYSTI_VERIFY_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mv_ctx mv_ctx;
typedef int32_t mv_status;

#define MV_OK 0
#define MV_E_INVALID_ARG (-1)
#define MV_E_HIP (-2)
#define MV_E_NO_DEVICE (-3)
#define MV_E_NO_COMMITTEE (-4)
#define MV_E_ALLOC (-5)

/* per-signature verdicts (ed25519_consensus::Error mapping) */
#define MV_SIG_OK 0
#define MV_SIG_INVALID 1       /* Error::InvalidSignature */
#define MV_SIG_MALFORMED_KEY 2 /* Error::MalformedPublicKey (A does not decode) */

/* per-block verdicts, in the error order of StatementBlock::verify (types.rs:315-376) */
#define MV_BLOCK_OK 0
#define MV_BLOCK_PARSE_ERROR 1             /* bincode::deserialize failed (data.rs:43-52) */
#define MV_BLOCK_DIGEST_MISMATCH 2         /* "Digest does not match" types.rs:327-332 */
#define MV_BLOCK_EPOCH_MISMATCH 3          /* types.rs:333-338 */
#define MV_BLOCK_UNKNOWN_AUTHOR 4          /* types.rs:339-342 */
#define MV_BLOCK_GENESIS 5                 /* types.rs:343-345 */
#define MV_BLOCK_SIG_INVALID 6             /* types.rs:346-348 */
#define MV_BLOCK_INCLUDE_UNKNOWN_AUTHORITY 7 /* types.rs:350-355 */
#define MV_BLOCK_INCLUDE_ROUND 8           /* types.rs:356-361 */
#define MV_BLOCK_VOTE_RANGE 9              /* first failing VoteRange (types.rs:363-370): end < start, */
                                           /* "offset_end_exclusive must be greater or equal ..." :441-446 */
#define MV_BLOCK_THRESHOLD_CLOCK 10        /* types.rs:371-374, threshold_clock.rs:12-35 */
#define MV_BLOCK_VOTE_RANGE_TOO_LONG 11    /* end - start >= 2^20, "Include is too large ..." :447-453 */
#define MV_BLOCK_VOTE_RANGE_END_TOO_LARGE 12 /* end >= 2^20, "offset_end_exclusive is too large ..." :454-458 */

/* per-entry WAL verdicts (WalReader::try_read, wal.rs:233-261; the reference panics on all but OK) */
#define MV_WAL_OK 0
#define MV_WAL_CRC_MISMATCH 1     /* "Crc mismatch, expected .., found .." wal.rs:250-257 */
#define MV_WAL_NONZERO_CRC_LEN0 2 /* "Non-zero crc at len 0" wal.rs:240-247 */
#define MV_WAL_BAD_LENGTH 3       /* len < 16 or the entry runs past its map: Bytes::slice panics, wal.rs:249 */

/* mv_config.flags */
#define MV_FLAG_NO_BATCH 1u /* host-buffer verify: never use the batch (random linear combination) path */
#define MV_FLAG_NO_COMB 2u  /* committee-key verifies: never use the per-key comb tables (ladder per signature) */
#define MV_FLAG_HOST_PARSE 4u /* mv_verify_blocks: parse the bincode on the host (block_codec.cpp), not on the GPU */
#define MV_FLAG_NO_ONLINE 8u  /* mv_verify_blocks: never use the resident online service (every call goes
                                 through the submission queue and launches its own kernels) */

/* Host-buffer verify calls of at least this many signatures per device take the batch path
 * (one combined equation + exact fallback); smaller ones verify every signature alone. */
#define MV_BATCH_MIN 4096u

typedef struct mv_config {
  uint32_t device_mask; /* bit i = use HIP device i; 0 = device 0 only */
  uint32_t max_batch;   /* items per device launch chunk; 0 = default (1<<20) */
  uint32_t flags;       /* MV_FLAG_* */
  uint32_t shards_per_device; /* 0/1 = one; k > 1: k logical shards (stream + buffers each) per device,
                                 host-buffer calls shard across them exactly as across GPUs */
} mv_config;

mv_status mv_create(const mv_config* cfg, mv_ctx** out);
void mv_destroy(mv_ctx* ctx);
const char* mv_last_error(const mv_ctx* ctx);
/* library version string, e.g. "mysti_verify 0.1 gfx950" */
const char* mv_version(void);

/* Committee: n authority keys (32-byte encodings) and stakes, committee epoch.
 * key_ok[i] (optional) receives 1 if key i decodes (VerificationKey::try_from). */
mv_status mv_set_committee(mv_ctx* ctx, const uint8_t* pks /* n x 32 */, const uint64_t* stakes, uint32_t n,
                           uint64_t epoch, uint8_t* key_ok /* n, may be NULL */);

/* Blake2b-256 of n byte strings buf[off[i] .. off[i]+len[i]) -> out[i] (32 B each). */
mv_status mv_blake2b256(mv_ctx* ctx, const uint8_t* buf, const uint64_t* off, const uint64_t* len, uint32_t n,
                        uint8_t* out /* n x 32 */);

/* ZIP-215 ed25519 verification of n signatures over 32-byte messages.
 * Keys: pk[i] if key_idx == NULL, else committee key key_idx[i] (pk must be NULL). */
mv_status mv_ed25519_verify(mv_ctx* ctx, const uint8_t* msg /* n x 32 */, const uint8_t* sig /* n x 64 */,
                            const uint8_t* pk /* n x 32 or NULL */, const uint32_t* key_idx /* n or NULL */,
                            uint32_t n, uint8_t* status /* n, MV_SIG_* */);

/* Page-locked host memory for verify inputs (hipHostMalloc, portable across the context's
 * devices). mv_ed25519_verify on inputs that are pinned (these, or any hipHostMalloc /
 * hipHostRegister memory) streams them in chunks whose H2D copies run beside the verification
 * of the previous chunk, instead of one pageable copy before the whole batch. Free with
 * mv_host_free. The Rust caller would receive network payloads into such buffers. */
mv_status mv_host_alloc(mv_ctx* ctx, uint64_t bytes, void** out);
void mv_host_free(mv_ctx* ctx, void* p);

/* RFC 8032 signing of n 32-byte messages with n 32-byte seeds -> pk (n x 32), sig (n x 64). */
mv_status mv_ed25519_sign(mv_ctx* ctx, const uint8_t* seed, const uint8_t* msg, uint32_t n, uint8_t* pk,
                          uint8_t* sig);

/* StatementBlock::verify on n bincode-serialized blocks buf[off[i] .. off[i]+len[i]).
 * status[i] = MV_BLOCK_*; msg_digest[i] = Blake2b-256(pre-image) (the signed message),
 * block_digest[i] = Blake2b-256(pre-image || signature); either digest array may be NULL.
 * Requires mv_set_committee. Concurrent callers are coalesced: a call joins a submission
 * queue, and a caller that finds no device pass running takes every queued call into one
 * pass (the online path: n - 1 peer tasks each with a block or two share a GPU round trip).
 * Several devices: the merged blocks are split into contiguous shards of about equal bytes.
 * Parameter order: status comes before the two (optional) digest arrays, unlike the draft in
 * SURVEY.md 8(b), so that the required outputs precede the NULL-able ones; `len` is u64 (blocks
 * are not bounded by 4 GiB in the type, and off/len share one type). */
mv_status mv_verify_blocks(mv_ctx* ctx, const uint8_t* buf, const uint64_t* off, const uint64_t* len, uint32_t n,
                           uint8_t* status, uint8_t* msg_digest, uint8_t* block_digest);

/* Submission-queue counters: mv_verify_blocks calls, and device passes that served them. */
mv_status mv_queue_stats(mv_ctx* ctx, uint64_t* calls, uint64_t* passes);

/* The resident online service (replaces the per-call device pass for the one-task-per-peer
 * traffic of NetworkSyncer, net_sync.rs:214-221 / synchronizer.rs:146-164): mv_verify_blocks
 * calls of <= 64 blocks and <= 128 KB of bincode, every block inside the device ingest's 10-KB
 * window (short and config-4-shape long blocks alike; MV_ONLINE_LONG=0 restricts the service to
 * calls averaging < MV_COMB_SPLIT_BYTES per block), are posted to a ring in page-locked memory
 * that a kernel resident on a highest-priority stream (a hardware queue of its own) polls; the
 * caller's thread spins on its
 * request's done word (no launch, no event, no wake-up per call). The kernel exits after
 * MV_ONLINE_IDLE_US (default 10,000) without work and is relaunched by the next call; calls it
 * does not take (more blocks or bytes, a block past the window, MV_FLAG_NO_ONLINE, MV_ONLINE=0)
 * go through the submission queue, and so does every call after the service has failed.
 * Verdicts and digests are those of the queue path. Counters: requests served by the service
 * and kernel launches it needed, summed over the context's devices. */
mv_status mv_online_stats(mv_ctx* ctx, uint64_t* requests, uint64_t* launches);

/* Host-only helper (no device needed): the shard plan of the multi-device paths -- cut[0..parts]
 * splits items [0, n) into contiguous shards of about equal total weight (block calls weigh a
 * block by its bincode bytes + 64). */
mv_status mv_shard_plan(const uint64_t* weights, uint64_t n, uint32_t parts, uint64_t* cut /* parts + 1 */);

/* Host-only helper (no device needed): the signed pre-image of one bincode block
 * (BlockDigest::digest_without_signature, crypto.rs:85-128). Returns the pre-image
 * length, or -1 if the bytes do not deserialize. `out` may be NULL to query the length. */
int64_t mv_block_preimage(const uint8_t* bincode, uint64_t len, uint8_t* out, uint64_t cap);

/* crc32fast::hash (CRC-32/ISO-HDLC) of n byte strings buf[off[i] .. off[i]+len[i]) -> out[i]. */
mv_status mv_crc32(mv_ctx* ctx, const uint8_t* buf, const uint64_t* off, const uint64_t* len, uint32_t n,
                   uint32_t* out /* n */);

/* WAL replay check: iterates the WAL image wal[0 .. size) as WalReader::iter_until does up to the
 * writer position end_pos (maps of 2^map_bits bytes: 24 in production, 16 under cfg(test),
 * wal.rs:95-103; 8 <= map_bits <= 30), checking every entry's crc32. Entries come out in
 * iteration order: pos[i] (WalPosition.start), tag[i], len[i] (payload bytes), status[i]
 * (MV_WAL_*). The iteration stops after the first entry whose status is not MV_WAL_OK (where
 * the reference panics). *count = the number of entries; only the first `cap` are written.
 * Bytes at or past `size` read as zero (the mapping's tail past the end of the file). */
mv_status mv_wal_verify(mv_ctx* ctx, const uint8_t* wal, uint64_t size, uint64_t end_pos, uint32_t map_bits,
                        uint64_t* pos, uint32_t* tag, uint32_t* len, uint8_t* status, uint64_t cap,
                        uint64_t* count);

/* Host-only helper: WalWriter::writev positions of n entries of payload_len[i] bytes written from
 * writer position `start` (an entry that would straddle a map starts at the next one); returns
 * the writer position after them. */
uint64_t mv_wal_layout(const uint64_t* payload_len, uint64_t n, uint32_t map_bits, uint64_t start,
                       uint64_t* pos /* n */);

/* Host-only helper: the Data<StatementBlock> byte strings inside received network frames
 * (Network::handle_read_stream, network.rs:400-447: a u32 big-endian size, then
 * bincode(NetworkMessage), network.rs:36-46; size 0 is a ping followed by 8 bytes). Lists the
 * blocks of every Blocks / RequestBlocksResponse message in buf[0, len) (u32 tag 1 or 3, u64
 * count, then u64 length + bytes per block, data.rs:67-96) as offsets into buf and lengths, in
 * stream order, for mv_verify_blocks on the same buffer (no copy of the bytes); the other
 * messages and pings are skipped unparsed. Stops before an incomplete trailing frame, and
 * *consumed (optional) = the bytes of the complete frames. Returns the number of blocks found
 * (the first `cap` written; cap 0 only counts), or -1 where the reference drops the connection:
 * a size above MAX_SIZE = 16 MiB (network.rs:216-221), a message tag above 4, or a block count
 * or length that runs past its frame (a bincode error, network.rs:454-457). */
int64_t mv_frame_blocks(const uint8_t* buf, uint64_t len, uint64_t* off, uint64_t* blen, uint64_t cap,
                        uint64_t* consumed);

/* ---- device-resident variants (inputs already in HBM of `device`) ----
 * Pointers are device pointers, 16-byte aligned; `stream` is a hipStream_t (NULL = the
 * library's stream for that device). They enqueue work and return without synchronising. */
mv_status mv_dev_ed25519_verify(mv_ctx* ctx, int device, const uint8_t* d_msg, const uint8_t* d_sig,
                                const uint8_t* d_pk, uint32_t n, uint8_t* d_status, void* stream);
/* Batch path on device buffers: verdicts identical to mv_dev_ed25519_verify. The combined
 * equation [8](-[sum z_i s_i]B + sum [z_i]R_i + sum [z_i k_i]A_i) == O with secret random
 * 127-bit z_i (BLAKE2b PRF keyed per context and call) is checked first, per sub-batch group
 * (mv_set_batch_groups); the signatures of every group whose equation fails are re-verified
 * individually on the same stream, so each verdict is exact (an invalid signature survives a
 * passing combination with probability <= 2^-127).
 * `d_pk` rows are indexed by item, or by `d_key_idx` (device array) when it is non-NULL; every
 * d_key_idx[i] must then be a row of d_pk (the library cannot bound-check device arrays).
 * Enqueues only; `d_batch_ok` (optional, device, 4 bytes) receives 1 if the combination held
 * (0 also when dense failures sent the call straight to per-signature verification, see
 * mv_batch_routes). The call makes `stream` wait only for the engine scratch slot it reuses;
 * MV_PREP_CHAIN=2 (mv_set_option) also orders its preparation after the previous call's. */
mv_status mv_dev_ed25519_verify_batch(mv_ctx* ctx, int device, const uint8_t* d_msg, const uint8_t* d_sig,
                                      const uint8_t* d_pk, const uint32_t* d_key_idx, uint32_t n,
                                      uint8_t* d_status, uint32_t* d_batch_ok, void* stream);
mv_status mv_dev_ed25519_sign(mv_ctx* ctx, int device, const uint8_t* d_seed, const uint8_t* d_msg, uint32_t n,
                              uint8_t* d_pk, uint8_t* d_sig, void* stream);
/* StatementBlock::verify on n bincode blocks already in HBM (Data::from_bytes + verify,
 * data.rs:43-52, types.rs:315-376): block i is d_buf[d_off[i] .. d_off[i] + d_len[i]). The
 * parse, the pre-image, both digests, the signature and the committee checks all run on the
 * device; verdicts as mv_verify_blocks. d_buf is 8-byte aligned, blocks do not overlap, and
 * 16 bytes past the end of every block are readable (pad the buffer); buf_bytes bounds the
 * blocks' extent in d_buf. d_msg_digest / d_block_digest (n x 32, 16-byte aligned) may be NULL.
 * Requires mv_set_committee. Enqueue only. */
mv_status mv_dev_verify_blocks(mv_ctx* ctx, int device, const uint8_t* d_buf, uint64_t buf_bytes,
                               const uint64_t* d_off, const uint64_t* d_len, uint32_t n, uint8_t* d_status,
                               uint8_t* d_msg_digest, uint8_t* d_block_digest, void* stream);

/* mv_wal_verify on a WAL image already in HBM (d_wal, 4-byte aligned); outputs are device arrays
 * of `cap` entries and *count is written on the host. Synchronises `stream` (the entry count is
 * data-dependent: the walk's per-map counts come back to the host before the crc pass). */
mv_status mv_dev_wal_verify(mv_ctx* ctx, int device, const uint8_t* d_wal, uint64_t size, uint64_t end_pos,
                            uint32_t map_bits, uint64_t* d_pos, uint32_t* d_tag, uint32_t* d_len, uint8_t* d_status,
                            uint64_t cap, uint64_t* count, void* stream);
/* crc32fast::hash of n strings of device buffer d_buf at d_off/d_len (device arrays) -> d_out. Enqueue only. */
mv_status mv_dev_crc32(mv_ctx* ctx, int device, const uint8_t* d_buf, const uint64_t* d_off, const uint64_t* d_len,
                       uint32_t n, uint32_t* d_out, void* stream);

/* ---- diagnostics (used by the test-suite) ---- */
/* Host-buffer batch-path counters since mv_create: batches tried, batches whose combined
 * equation failed (and were re-verified signature by signature). */
mv_status mv_batch_stats(mv_ctx* ctx, uint64_t* batches, uint64_t* fallbacks);
/* batch counters: out[0] batches, out[1] batches whose combined equation failed in some
 * sub-batch, out[2] sub-batch equations checked, out[3] sub-batch equations that failed
 * (each re-verified signature by signature). Device-API calls are counted once complete. */
mv_status mv_batch_counters(mv_ctx* ctx, uint64_t* out /* 4 */);
/* Routes of batch-path calls under the adaptive policy (config 3, net_sync.rs:352-361: a peer
 * that keeps sending bad signatures): out[0] batches checked by a combined equation (as
 * mv_batch_stats), out[1] batches sent straight to per-signature verification because the
 * failures were dense, out[2] dense failures seen (a guarded batch with at least half of its
 * sub-batch equations failed). Device-API calls are counted once complete. */
mv_status mv_batch_routes(mv_ctx* ctx, uint64_t* out /* 3 */);
/* Sub-batch equations per batch-path call: the batch is cut into groups of whole 1024-signature
 * chunks, each with its own combined equation, and a failed equation re-verifies only its group.
 * groups = 0 (default): adaptive -- 1 group per batch; after a batch whose equation failed,
 * the next 64 batches are cut into 8; after a guarded batch in which at least half of the
 * equations failed (dense failures: the combined check is wasted work), the next batches are
 * verified signature by signature, each counting its invalid signatures, until one holds fewer
 * than 4 (then the guarded equation again). groups = 1..16 fixes the count and disables the
 * dense-failure route. Every call clears the guard. Verdicts never depend on it. */
mv_status mv_set_batch_groups(mv_ctx* ctx, uint32_t groups);
/* Stage timing: when enabled, every call records HIP events on its stream around its
 * stages: batch path 0..5 (prep, sort, bucket, reduce, final, fallback), block pipeline
 * 6..9 (parse, hash, verify = comb/ladder verify when the batch path is not taken, verdict),
 * WAL replay 10..11 (walk = the per-map header walk, crc = the entry crc pass).
 * mv_stage_times waits for the recorded calls and returns the summed device ms per stage and
 * the number of calls measured per stage; reset != 0 clears the sums. */
#define MV_NSTAGES 12
mv_status mv_set_stage_timing(mv_ctx* ctx, int enable);
mv_status mv_stage_times(mv_ctx* ctx, double* ms /* MV_NSTAGES or NULL */, uint64_t* calls /* MV_NSTAGES or NULL */,
                         int reset);
/* Runtime switches (MV_ONLINE, MV_COMB_QUAD, MV_ONLINE_IDLE_US, ...). The library
 * reads every switch from the environment once, at mv_create -- as the reference reads its env
 * knobs at start-up (validator.rs:104-119) -- and never per call. mv_set_option changes one
 * afterwards, between calls (no call on ctx in flight); name is the environment name and value
 * an integer (0 / 1 for on/off switches). Unknown names, and the switches consumed by
 * mv_create (MV_PASS_SETS, MV_GUARD_GROUPS, MV_BASE_GROUPS), are MV_E_INVALID_ARG. No switch
 * changes a verdict, digest or crc. */
mv_status mv_set_option(mv_ctx* ctx, const char* name, int64_t value);
mv_status mv_get_option(mv_ctx* ctx, const char* name, int64_t* value);
/* Runs field/scalar primitive `op` on n lane inputs (16 words each) -> 16 words each (host buffers). */
mv_status mv_selftest(mv_ctx* ctx, int op, const uint32_t* in, uint32_t n, uint32_t* out);

#ifdef __cplusplus
}
#endif
#endif /* MYSTI_VERIFY_H */
