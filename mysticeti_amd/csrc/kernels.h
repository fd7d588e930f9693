// Host-side launchers for kernels.hip (internal to libmysti_verify.so).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace mvk {
// The runtime switches. Read from the environment once, at mv_create
// (knobs_from_env in engine.cpp, the only getenv in the library), and stored in the context; the
// diagnostics entry point mv_set_option changes one between calls (the tests select forms that
// way). None changes a verdict, digest or crc. Launchers that choose between kernel forms take
// the context's Knobs as their first argument.
struct Knobs {
  // block path (engine.cpp)
  int64_t blk_pipe = 1;                  // MV_BLK_PIPE: batch-size block calls in two halves on two streams
  int64_t comb_split_bytes = 2048;       // MV_COMB_SPLIT_BYTES: bytes per block from which the split comb path runs
  int64_t hash_in_comb = 1;              // MV_HASH_IN_COMB: online passes hash inside k_verify_comb16
  int64_t ingest_in_comb = 1;            // MV_INGEST_IN_COMB: ... and parse there
  int64_t verdict_fused = 1;             // MV_VERDICT_FUSED: the block verdict inside the comb kernels
  int64_t blk_chunk_bytes = 256ll << 20;  // MV_BLK_CHUNK_BYTES: bytes per host-buffer block chunk
  int64_t pack_threads = 0;              // MV_PACK_THREADS: host threads packing a chunk (0: min(8, cores))
  int64_t blk_trace = 0;                 // MV_BLK_TRACE: host-side timing lines on stderr
  int64_t blk_zerocopy = 1ll << 20;      // MV_BLK_ZEROCOPY: passes up to this size read pinned staging
  int64_t pass_spin = 0;                 // MV_PASS_SPIN: the pass owner polls its event
  int64_t pass_sets = 2;                 // MV_PASS_SETS: submission-queue pass sets (2 .. 4)
  int64_t q_linger_us = 50;              // MV_Q_LINGER_US
  int64_t q_spin_us = 0;                 // MV_Q_SPIN_US
  // the resident online service
  int64_t online = 1;                    // MV_ONLINE: small block calls take the service
  int64_t online_long = 1;               // MV_ONLINE_LONG: long blocks take it too
  int64_t online_prio = 1;               // MV_ONLINE_PRIO: the service stream at the highest priority (its own queue)
  int64_t online_wgs = 0;                // MV_ONLINE_WGS: resident workgroups (0: = CUs)
  int64_t online_idle_us = 10000;        // MV_ONLINE_IDLE_US: the launch ends after this long idle
  int64_t online_trace = 0;              // MV_ONLINE_TRACE: per-stage means on stderr at release
  int64_t online_debug = 0;              // MV_ONLINE_DEBUG: launch lines, long waits on stderr
  int64_t online_inject = 0;             // MV_ONLINE_INJECT: fault injection (tests): launches fail
  int64_t online_spinners = 0;           // MV_ONLINE_SPINNERS: callers spinning on their verdict (0: 1/4 of the CPU share)
  // signature path
  int64_t stream_chunk_log2 = 17;        // MV_STREAM_CHUNK_LOG2: signatures per copy chunk
  int64_t guard_groups = 8;              // MV_GUARD_GROUPS: sub-batches while guarded
  int64_t base_groups = 1;               // MV_BASE_GROUPS: sub-batches when not guarded
  double stream_fracs[8] = {0.7, 0.3};   // MV_STREAM_FRACS: the streamed batches' shares
  int n_stream_fracs = 2;
  // kernel forms (the launchers)
  int64_t no_key_agg = 0;                // MV_NO_KEY_AGG: committee A terms as bucket entries
  int64_t reduce_quad = 16384;           // MV_REDUCE_QUAD: quad-reduce threshold
  int64_t bv_seg = -1;                   // MV_BV_SEG: bucket segment length (-1: measured best)
  int64_t b2q_ns = 0;                    // MV_B2Q_NS: strings per quad in k_b2_quad (2: interleaved)
  int64_t b2_lane = 1;                   // MV_B2_LANE: batch-size BLAKE2b one lane per string
  int64_t comb_quad = -1;                // MV_COMB_QUAD: force k_verify_comb16 (1) / k_verify_comb (0)
  int64_t ingest_lane = 0;               // MV_INGEST_LANE: the lane-per-block ingest kernel
  int64_t verify_occ = 2;                // MV_VERIFY_OCC: k_verify's waves per SIMD (1, 2, 3)
  int64_t reduce_rows = 1024;            // MV_REDUCE_ROWS: reduction levels of <= this many elements a wave each (0: none)
  int64_t fine_lds = 1;                  // MV_FINE_LDS: the fine sort staged in registers + LDS (coalesced stores)
  int64_t scatter_lds = 1;               // MV_SCATTER_LDS: the partition scatter staged in LDS (coalesced stores)
  int64_t final_rows = 1;                // MV_FINAL_ROWS: k_bv_final's Horner with one DPP row per coordinate
  int64_t bucket_bal = 1;                // MV_BUCKET_BAL: equal entries per bucket-kernel lane (>1: entries per lane)
  int64_t prep_chain = 1;                // MV_PREP_CHAIN: a batch's k_bv_prep starts after the previous batch's
                                         // (1: on the engine's streams; 2: on callers' streams too)
  int64_t blk_walk = 1;                  // MV_BLK_WALK: batch-size block calls in one pass over the bincode (k_block_walk); 0: staged pre-image
};

size_t verify_scratch_bytes(uint32_t n);
size_t btable_bytes();
hipError_t launch_btable_init(void* d_btab, hipStream_t s);
hipError_t launch_verify(const Knobs& kn, const uint8_t* msg, const uint8_t* sig, const uint8_t* pk, const uint32_t* key_idx,
                         uint32_t n, const void* btab, void* scratch, uint8_t* status, hipStream_t s,
                         const uint32_t* skip = nullptr, uint32_t skip_group = 0, const void* prep_pts = nullptr,
                         const void* prep_comb = nullptr);
// skip (optional, device): per-group flags; the signatures of group g = i / skip_group
// (skip_group a multiple of 256; 0 = one group) are not verified when skip[g] != 0.
// prep_pts (the batch path's fallback): R and A as k_bv_prep decoded them (A from the comb
// tables prep_comb when it was summed per key), and prep's nonzero statuses kept.
// *count = the number of items of status[0..n) equal to MV_SIG_INVALID; status 16-byte aligned
hipError_t launch_count_rejects(const uint8_t* status, uint32_t n, uint32_t* count, hipStream_t s);
hipError_t launch_sign(const uint8_t* seed, const uint8_t* msg, uint32_t n, const void* btab, uint8_t* pk,
                       uint8_t* sig, hipStream_t s);
hipError_t launch_blake2b(const Knobs& kn, const uint8_t* buf, const uint64_t* off, const uint64_t* len, uint32_t n, uint8_t* out,
                          hipStream_t s);
hipError_t launch_block_hash(const Knobs& kn, const uint8_t* buf, const uint64_t* off, const uint64_t* len, uint32_t n,
                             uint8_t* msg_out, uint8_t* dig_out, hipStream_t s);
// blake2b_quad.hip: the same two hashes with four lanes per string (launch_blake2b /
// launch_block_hash route to them; at batch size they route on to blake2b_lane.hip)
hipError_t launch_blake2b_quad(const Knobs& kn, const uint8_t* buf, const uint64_t* off, const uint64_t* len, uint32_t n, uint8_t* out,
                               hipStream_t s);
hipError_t launch_block_hash_quad(const Knobs& kn, const uint8_t* buf, const uint64_t* off, const uint64_t* len, uint32_t n,
                                  uint8_t* msg_out, uint8_t* dig_out, hipStream_t s);
// blake2b_lane.hip: one lane per string (batch-size calls; the quad launchers route to it)
hipError_t launch_blake2b_lane(const uint8_t* buf, const uint64_t* off, const uint64_t* len, uint32_t n, uint8_t* out,
                               hipStream_t s);
hipError_t launch_block_hash_lane(const uint8_t* buf, const uint64_t* off, const uint64_t* len, uint32_t n,
                                  uint8_t* msg_out, uint8_t* dig_out, hipStream_t s);
hipError_t launch_selftest(int op, const uint32_t* in, uint32_t n, const void* btab, uint32_t* out, hipStream_t s);
// batch.hip: random-linear-combination batch verify with exact on-device fallback.
// The batch is cut into `groups` sub-batches (1..BATCH_MAX_GROUPS, whole 1024-signature
// chunks, batch_group_size signatures each), one combined equation per group.
// key = 32-byte secret + 64-bit call counter (the z_i PRF key); *flag_out receives the
// device address of the flag words: [0] = 1 if every group's equation held, [1 + g] = 1
// if group g's held. ev (optional): BATCH_STAGES + 1 events, recorded before the first
// stage and after each stage.
struct ChunkGate {
  const hipEvent_t* ready;
  uint32_t n;
  const uint32_t* end;
};
constexpr int BATCH_STAGES = 6;  // prep, sort, bucket, reduce, final, fallback
constexpr int BATCH_MAX_GROUPS = 16;
size_t batch_scratch_bytes(uint32_t n, uint32_t groups);
uint32_t batch_group_size(uint32_t n, uint32_t groups);
hipError_t launch_verify_batch(const Knobs& kn, const uint8_t* msg, const uint8_t* sig, const uint8_t* pk, const uint32_t* key_idx,
                               uint32_t n, uint32_t groups, const uint32_t key[10], const void* btab,
                               void* bscratch, void* vscratch, uint8_t* status, hipStream_t s,
                               uint32_t** flag_out, hipEvent_t* ev = nullptr, const void* comb_a = nullptr,
                               const uint8_t* key_ok = nullptr, uint32_t n_keys = 0, const void* comb_b = nullptr,
                               const struct ChunkGate* gate = nullptr, const hipEvent_t* chain = nullptr);
// chain (optional, unchunked calls): k_bv_prep waits for chain[0] (may be null) and chain[1]
// is recorded after it, so consecutive batches on different streams run their preparations
// one after another and each overlaps the previous batches' narrow tails (sort, reduce, final)
// instead of all starting together and leaving the tails to run side by side.
// gate (optional): the inputs arrive in chunks (H2D copies on another stream). Chunk c =
// signatures [end[c - 1], end[c]) (ends multiples of 256 except the last = n); k_bv_prep runs
// chunk by chunk on s, each launch after hipStreamWaitEvent on ready[c].
// comb_b (required): the comb table of B (mv_create), for the -[sum z s]B term.
// comb_a / key_ok (optional, with key_idx): the committee's comb tables (comb.hip, tables of
// -A) and per-key decode flags; k_bv_prep then reads each signature's A from entry [0][1]
// of its key's table instead of decoding A (the key was decoded once, at mv_set_committee).
// n_keys (committee size, <= 512) > 0 also sums A's term per key: sum_b [c_b] A_b on the
// comb tables replaces the 16 A bucket entries per signature.
// comb.hip: per-key comb tables C[i][j] = [j 256^i](+-P) and the committee-key verify.
// enc == nullptr builds the table of B; negate = 1 stores -P (committee keys).
size_t comb_table_bytes(uint32_t nbases);
hipError_t launch_comb_init(const uint8_t* enc, uint32_t nb, int negate, void* tab, uint8_t* ok, hipStream_t s);
// the block verdict (block_verdict.h) fused into a committee signature kernel's last step on
// the online block path, which then writes status[] instead of the signature status: one
// launch less. Null: signature status only.
struct BlockVerdictOut {
  const uint32_t* facts;
  const uint8_t* claimed;
  uint8_t* msg_digest;
  uint8_t* digest;
  uint8_t* status;
};
// the block hash folded into the online committee verify (k_verify_comb16): the staged
// pre-images P || sig in, both digests out (msg_digest is then the kernel's msg input)
struct BlockHashIn {
  const uint8_t* stage;
  const uint64_t* pre_off;
  const uint64_t* pre_len;
  uint8_t* msg_digest;
  uint8_t* digest;
};
// the block ingest folded into the online committee verify too (k_verify_comb16 parses its own
// blocks first, one wave per block): bincode in, everything launch_block_parse writes out
struct BlockIngestIn {
  const uint8_t* buf;
  const uint64_t* off;
  const uint64_t* len;
  const uint64_t* stakes;
  uint32_t n_auth;
  uint64_t epoch, quorum_thr;
  uint8_t* stage;
  uint64_t* pre_off;
  uint64_t* pre_len;
  uint8_t* sig;
  uint32_t* key_idx;
  uint32_t* facts;
  uint8_t* claimed;
};
// The resident online service (comb.hip k_online): one kernel that stays on the GPU while
// online traffic flows and runs each mv_verify_blocks request of <= ONLINE_MAX_BLOCKS short
// blocks as k_verify_comb16's workgroups would (ingest, both digests, challenge, comb sums,
// verdict), with no launch and no event per request.
//   host     writes request q's input (offsets, lengths, bincode) into ring slot q % SLOTS of
//            page-locked memory and its descriptor, then seq = q + 1; ctl.tail >= q + 1
//   poller   workgroup 0 polls ctl.tail, copies the input of every request whose seq is set
//            into the slot's HBM scratch (one pass for all of them) and appends the request's
//            4-block jobs to a job ring in HBM: the only PCIe reads on the request's path
//   workers  workgroups 1.. each hold a ticket (one atomic add on the ring's head) and start the
//            job as soon as the ring's tail passes it, run it from HBM, copy its blocks' digests
//            and verdicts to the slot's page-locked output; the request's last job stores
//            ctl.done[slot] = q + 1 (system-scope release after the outputs)
// The poller ends the launch (quit) after idle_ticks without a request, on ctl.stop, or after
// max_ticks; workers leave when they see quit. A launch starts by discarding tickets of the
// previous launch's workers (head = tail) before any worker takes one (epoch handshake).
// The slot's HBM scratch layout is fixed (below), so a descriptor is 16 bytes.
#ifndef MV_ONLINE_SLOTS
#define MV_ONLINE_SLOTS 128
#endif
constexpr uint32_t ONLINE_SLOTS = MV_ONLINE_SLOTS;  // request ring (a multiple of 64)
constexpr uint32_t ONLINE_MAX_BLOCKS = 64;  // 16 jobs per request
constexpr uint32_t ONLINE_JOBS = 16 * ONLINE_SLOTS;  // job ring (>= SLOTS x 16)
constexpr uint32_t ONLINE_MAX_WGS = 256;    // resident workgroups at most (the poller + workers)
constexpr uint32_t ONLINE_WG_LEFT = 0x80000000u;
constexpr uint64_t ONLINE_EXIT_STOP = 1, ONLINE_EXIT_IDLE = 2, ONLINE_EXIT_MAX = 3;
constexpr size_t ONLINE_IN_CAP = 128u << 10;  // bincode bytes per request
constexpr size_t online_al(size_t x) { return (x + 255) & ~(size_t)255; }
constexpr size_t ONLINE_IN_STRIDE = online_al(16 * ONLINE_MAX_BLOCKS + ONLINE_IN_CAP + 64);  // off | len | bincode
constexpr size_t ONLINE_OUT_STRIDE = online_al(65 * ONLINE_MAX_BLOCKS);  // md[64][32] | bd[64][32] | status[64]
// slot scratch (HBM): in | out | stage | pre_off | pre_len | sig | key_idx | facts | claimed | sst
constexpr size_t ONLINE_O_OUT = ONLINE_IN_STRIDE;
constexpr size_t ONLINE_O_STAGE = ONLINE_O_OUT + ONLINE_OUT_STRIDE;
constexpr size_t ONLINE_O_POFF = ONLINE_O_STAGE + online_al(ONLINE_IN_CAP + 4096);
constexpr size_t ONLINE_O_PLEN = ONLINE_O_POFF + online_al(8 * ONLINE_MAX_BLOCKS);
constexpr size_t ONLINE_O_SIG = ONLINE_O_PLEN + online_al(8 * ONLINE_MAX_BLOCKS);
constexpr size_t ONLINE_O_KIDX = ONLINE_O_SIG + online_al(64 * ONLINE_MAX_BLOCKS);
constexpr size_t ONLINE_O_FACTS = ONLINE_O_KIDX + online_al(4 * ONLINE_MAX_BLOCKS);
constexpr size_t ONLINE_O_CLAIMED = ONLINE_O_FACTS + online_al(4 * ONLINE_MAX_BLOCKS);
constexpr size_t ONLINE_O_SST = ONLINE_O_CLAIMED + online_al(32 * ONLINE_MAX_BLOCKS);
constexpr size_t ONLINE_SCR_STRIDE = ONLINE_O_SST + online_al(ONLINE_MAX_BLOCKS);
// the wave-parallel ingest's LDS window per block (ingest_dev.h IG_WIN): longer blocks parse on
// one lane, so the online service leaves them to the queue
constexpr uint32_t INGEST_WINDOW_BYTES = 10240;
struct OnlineReq {
  uint64_t seq;         // request number + 1 once the slot's input and n are written (release)
  uint32_t n;           // blocks; 0 = a void request (completed without work)
  uint32_t copy_bytes;  // input bytes of the slot (offsets, lengths, bincode + 16 zero bytes)
};
struct OnlineCtl {
  uint64_t tail;  // requests published so far
  uint64_t stop;  // nonzero: end the launch when idle
  uint64_t done[ONLINE_SLOTS];
  // the kernel's wall clock at: the poller sees the request, its jobs are in the ring, its first
  // job starts, its last job is done; then job 0's barrier 0 (ingest done), B rows done, S done,
  // R decoded, barrier 1, verdict written, outputs fenced, digests done, k published (comb.hip
  // comb16_wg; diagnostics: MV_ONLINE_TRACE sums them)
  uint64_t trace[ONLINE_SLOTS][14];
  // liveness (plain system-scope stores, read by the host's bounded stop): the workgroup's launch
  // number while it runs, | ONLINE_WG_LEFT once it has left; the poller's exit reason and its
  // ring words at exit (ready, jobs_head, jobs_tail)
  uint32_t wg[ONLINE_MAX_WGS];
  uint64_t exit_why, exit_ready, exit_head, exit_tail;
};
struct OnlineDev {
  unsigned long long ready;      // requests moved to HBM by the poller
  unsigned long long jobs_head;  // next ticket
  unsigned long long jobs_tail;  // jobs appended
  uint32_t quit, epoch;          // quit: workers leave; epoch: the launch whose poller is set up
  uint32_t n[ONLINE_SLOTS];
  uint32_t jobs_done[ONLINE_SLOTS];
  unsigned long long moved[ONLINE_SLOTS];  // request + 1 last moved from each slot (the poller's)
  unsigned long long jobs[ONLINE_JOBS];  // (request << 8) | job
  uint64_t sink[2 * 1024];               // 16 B per poller thread: where its copy lanes past the end go
};
struct OnlineArgs {
  OnlineCtl* ctl;                 // page-locked (device view)
  const OnlineReq* reqs;          // page-locked ring of descriptors
  OnlineDev* dev;                 // HBM
  const uint8_t* in_host;         // page-locked inputs, ONLINE_IN_STRIDE per slot
  uint8_t* out_host;              // page-locked outputs, ONLINE_OUT_STRIDE per slot
  uint8_t* scr;                   // HBM scratch, ONLINE_SCR_STRIDE per slot
  const void* combB;
  const void* combA;
  const uint8_t* key_ok;
  const uint8_t* pk;              // committee keys (32 B each)
  const uint64_t* stakes;
  uint64_t epoch, quorum_thr;     // the committee's
  uint32_t n_auth;
  uint32_t launch;                // launch number (the epoch handshake)
  uint64_t idle_ticks, max_ticks;
};
hipError_t launch_online(const OnlineArgs& a, uint32_t grid, hipStream_t s);
hipError_t launch_verify_comb(const Knobs& kn, const uint8_t* msg, const uint8_t* sig, const uint8_t* pk, const uint32_t* key_idx,
                              uint32_t n, const void* combB, const void* combA, const uint8_t* key_ok,
                              uint8_t* status, hipStream_t s, const BlockVerdictOut* bv = nullptr,
                              const BlockHashIn* hin = nullptr, const BlockIngestIn* ing = nullptr);
// whether launch_verify_comb takes the short-chain kernel (the one that can fold the hash in)
bool comb_short_chain(const Knobs& kn, uint32_t n);
// the comb verify split in two, for small batches of long blocks: k_hash_comb_pre is
// launch_block_hash plus, on workgroups of their own, the signature-only terms (R decoded ->
// rbuf, -[s]B -> sbuf, 144 B per signature each, flags: bit 0 s < l, bit 1 R decodes);
// k_comb_post adds the message-dependent [k]A and tests [8](R - R') = O
hipError_t launch_hash_comb_pre(const uint8_t* stage, const uint64_t* poff, const uint64_t* plen, uint32_t n,
                                uint8_t* md, uint8_t* bd, const uint8_t* sig, const void* combB, void* rbuf,
                                void* sbuf, uint8_t* qflags, hipStream_t s);
hipError_t launch_comb_post(const uint8_t* msg, const uint8_t* sig, const uint8_t* pk, const uint32_t* key_idx,
                            uint32_t n, const void* combA, const uint8_t* key_ok, const void* rbuf,
                            const void* sbuf, const uint8_t* qflags, uint8_t* status, hipStream_t s,
                            const BlockVerdictOut* bv = nullptr);
// ingest.hip: device-side bincode parse + pre-image staging, and the final block verdict
hipError_t launch_block_parse(const Knobs& kn, const uint8_t* buf, const uint64_t* off, const uint64_t* len, uint32_t n,
                              const uint64_t* stakes, uint32_t n_auth, uint64_t epoch, uint64_t quorum_thr,
                              uint8_t* stage, uint64_t* pre_off, uint64_t* pre_len, uint8_t* sig, uint32_t* key_idx,
                              uint32_t* facts, uint8_t* claimed, hipStream_t s);
// block_walk.hip: launch_block_parse's outputs (but no staged pre-image) and both digests in
// ONE pass over the bincode, one lane per block; committees of <= 512 authorities
hipError_t launch_block_walk(const uint8_t* buf, const uint64_t* off, const uint64_t* len, uint32_t n,
                             const uint64_t* stakes, uint32_t n_auth, uint64_t epoch, uint64_t quorum_thr,
                             uint8_t* sig, uint32_t* key_idx, uint32_t* facts, uint8_t* claimed, uint8_t* md,
                             uint8_t* bd, hipStream_t s);
// sig[i]'s s := 2^256 - 1 (outside the batch equation) for every parsed block whose computed
// digest differs from its claimed one
hipError_t launch_block_digest_gate(const uint8_t* claimed, const uint8_t* digest, const uint32_t* facts, uint32_t n,
                                    uint8_t* sig, hipStream_t s);
// status in the types.rs order; zeroes both digests of blocks that do not deserialize
hipError_t launch_block_verdict(const uint32_t* facts, const uint8_t* claimed, uint8_t* msg_digest, uint8_t* digest,
                                const uint8_t* sig_status, uint32_t n, uint8_t* status, hipStream_t s);
// wal.hip: crc32fast::hash on the GPU and the WAL replay walk. `tables`
// (wal_table_words() words, built by wal_build_tables on the host) stay resident per device.
// cus = compute units (sizes the persistent crc grids).
size_t wal_table_words();
void wal_build_tables(uint32_t* out);
hipError_t launch_crc32(const uint8_t* buf, const uint64_t* off, const uint64_t* len, uint32_t n,
                        const uint32_t* tables, uint32_t* out, int cus, hipStream_t s);
// one lane per map: records (position | walk status << 60) of map m at rec[m * cap_pm ..], the
// record count (may exceed cap_pm: nothing past it is stored) and how the iteration leaves the map.
// moff (optional, a second walk): map m's records at rec[moff[m] ..], mcount[m] of them (the
// first walk's counts, read by the kernel)
constexpr uint8_t WAL_MAP_EMPTY = 0, WAL_MAP_NEXT = 1, WAL_MAP_END = 2, WAL_MAP_BAD = 3;
hipError_t launch_wal_walk(const uint8_t* img, uint64_t size, uint64_t end_pos, uint32_t map_bits, uint32_t nmaps,
                           uint32_t cap_pm, const uint64_t* moff, unsigned long long* rec, uint32_t* mcount,
                           uint8_t* mflag, hipStream_t s);
hipError_t launch_wal_compact(const unsigned long long* rec, uint32_t cap_pm, const uint32_t* mcount,
                              const uint64_t* moff, uint32_t nmaps, unsigned long long* ent, hipStream_t s);
// one wave per entry: header, payload crc, verdict (MV_WAL_*); *first_fail = min failing index
hipError_t launch_wal_crc(const uint8_t* img, uint64_t size, const unsigned long long* ent, uint64_t total,
                          const uint32_t* tables, uint64_t* out_pos, uint32_t* out_tag, uint32_t* out_len,
                          uint8_t* out_status, uint64_t cap, unsigned long long* first_fail, int cus, hipStream_t s);
}  // namespace mvk
