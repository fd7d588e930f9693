//! Raw declarations of include/mysti_verify.h (the C ABI of libmysti_verify.so).
//! Each entry point names the reference interface it replaces in the header's comments.
#![allow(non_camel_case_types)]
use std::os::raw::{c_char, c_void};

#[repr(C)]
pub struct mv_ctx {
    _p: [u8; 0],
}

#[repr(C)]
#[derive(Default, Clone, Copy)]
pub struct mv_config {
    pub device_mask: u32,
    pub max_batch: u32,
    pub flags: u32,
    pub shards_per_device: u32,
}

pub const MV_OK: i32 = 0;
pub const MV_E_INVALID_ARG: i32 = -1;
pub const MV_E_HIP: i32 = -2;
pub const MV_E_NO_DEVICE: i32 = -3;
pub const MV_E_NO_COMMITTEE: i32 = -4;
pub const MV_E_ALLOC: i32 = -5;

pub const MV_SIG_OK: u8 = 0;
pub const MV_SIG_INVALID: u8 = 1;
pub const MV_SIG_MALFORMED_KEY: u8 = 2;

pub const MV_BLOCK_OK: u8 = 0;
pub const MV_BLOCK_PARSE_ERROR: u8 = 1;
pub const MV_BLOCK_DIGEST_MISMATCH: u8 = 2;
pub const MV_BLOCK_EPOCH_MISMATCH: u8 = 3;
pub const MV_BLOCK_UNKNOWN_AUTHOR: u8 = 4;
pub const MV_BLOCK_GENESIS: u8 = 5;
pub const MV_BLOCK_SIG_INVALID: u8 = 6;
pub const MV_BLOCK_INCLUDE_UNKNOWN_AUTHORITY: u8 = 7;
pub const MV_BLOCK_INCLUDE_ROUND: u8 = 8;
pub const MV_BLOCK_VOTE_RANGE: u8 = 9;
pub const MV_BLOCK_THRESHOLD_CLOCK: u8 = 10;
pub const MV_BLOCK_VOTE_RANGE_TOO_LONG: u8 = 11;
pub const MV_BLOCK_VOTE_RANGE_END_TOO_LARGE: u8 = 12;

pub const MV_WAL_OK: u8 = 0;
pub const MV_WAL_CRC_MISMATCH: u8 = 1;
pub const MV_WAL_NONZERO_CRC_LEN0: u8 = 2;
pub const MV_WAL_BAD_LENGTH: u8 = 3;

pub const MV_FLAG_NO_BATCH: u32 = 1;
pub const MV_FLAG_NO_COMB: u32 = 2;
pub const MV_FLAG_HOST_PARSE: u32 = 4;
pub const MV_FLAG_NO_ONLINE: u32 = 8;
pub const MV_BATCH_MIN: u32 = 4096;
pub const MV_NSTAGES: usize = 12;

extern "C" {
    pub fn mv_create(cfg: *const mv_config, out: *mut *mut mv_ctx) -> i32;
    pub fn mv_destroy(ctx: *mut mv_ctx);
    pub fn mv_last_error(ctx: *const mv_ctx) -> *const c_char;
    pub fn mv_version() -> *const c_char;
    pub fn mv_set_committee(ctx: *mut mv_ctx, pks: *const u8, stakes: *const u64, n: u32, epoch: u64,
                            key_ok: *mut u8) -> i32;
    pub fn mv_blake2b256(ctx: *mut mv_ctx, buf: *const u8, off: *const u64, len: *const u64, n: u32,
                         out: *mut u8) -> i32;
    pub fn mv_ed25519_verify(ctx: *mut mv_ctx, msg: *const u8, sig: *const u8, pk: *const u8,
                             key_idx: *const u32, n: u32, status: *mut u8) -> i32;
    pub fn mv_host_alloc(ctx: *mut mv_ctx, bytes: u64, out: *mut *mut c_void) -> i32;
    pub fn mv_host_free(ctx: *mut mv_ctx, p: *mut c_void);
    pub fn mv_ed25519_sign(ctx: *mut mv_ctx, seed: *const u8, msg: *const u8, n: u32, pk: *mut u8,
                           sig: *mut u8) -> i32;
    pub fn mv_verify_blocks(ctx: *mut mv_ctx, buf: *const u8, off: *const u64, len: *const u64, n: u32,
                            status: *mut u8, msg_digest: *mut u8, block_digest: *mut u8) -> i32;
    pub fn mv_block_preimage(bincode: *const u8, len: u64, out: *mut u8, cap: u64) -> i64;
    pub fn mv_queue_stats(ctx: *mut mv_ctx, calls: *mut u64, passes: *mut u64) -> i32;
    pub fn mv_online_stats(ctx: *mut mv_ctx, requests: *mut u64, launches: *mut u64) -> i32;
    pub fn mv_shard_plan(weights: *const u64, n: u64, parts: u32, cut: *mut u64) -> i32;
    pub fn mv_crc32(ctx: *mut mv_ctx, buf: *const u8, off: *const u64, len: *const u64, n: u32,
                    out: *mut u32) -> i32;
    pub fn mv_wal_verify(ctx: *mut mv_ctx, wal: *const u8, size: u64, end_pos: u64, map_bits: u32,
                         pos: *mut u64, tag: *mut u32, len: *mut u32, status: *mut u8, cap: u64,
                         count: *mut u64) -> i32;
    pub fn mv_wal_layout(payload_len: *const u64, n: u64, map_bits: u32, start: u64, pos: *mut u64) -> u64;
    pub fn mv_frame_blocks(buf: *const u8, len: u64, off: *mut u64, blen: *mut u64, cap: u64,
                           consumed: *mut u64) -> i64;
    pub fn mv_dev_ed25519_verify(ctx: *mut mv_ctx, device: i32, d_msg: *const u8, d_sig: *const u8,
                                 d_pk: *const u8, n: u32, d_status: *mut u8, stream: *mut c_void) -> i32;
    pub fn mv_dev_ed25519_verify_batch(ctx: *mut mv_ctx, device: i32, d_msg: *const u8, d_sig: *const u8,
                                       d_pk: *const u8, d_key_idx: *const u32, n: u32, d_status: *mut u8,
                                       d_batch_ok: *mut u32, stream: *mut c_void) -> i32;
    pub fn mv_dev_ed25519_sign(ctx: *mut mv_ctx, device: i32, d_seed: *const u8, d_msg: *const u8, n: u32,
                               d_pk: *mut u8, d_sig: *mut u8, stream: *mut c_void) -> i32;
    pub fn mv_dev_verify_blocks(ctx: *mut mv_ctx, device: i32, d_buf: *const u8, buf_bytes: u64,
                                d_off: *const u64, d_len: *const u64, n: u32, d_status: *mut u8,
                                d_msg_digest: *mut u8, d_block_digest: *mut u8, stream: *mut c_void) -> i32;
    pub fn mv_dev_wal_verify(ctx: *mut mv_ctx, device: i32, d_wal: *const u8, size: u64, end_pos: u64,
                             map_bits: u32, d_pos: *mut u64, d_tag: *mut u32, d_len: *mut u32,
                             d_status: *mut u8, cap: u64, count: *mut u64, stream: *mut c_void) -> i32;
    pub fn mv_dev_crc32(ctx: *mut mv_ctx, device: i32, d_buf: *const u8, d_off: *const u64, d_len: *const u64,
                        n: u32, d_out: *mut u32, stream: *mut c_void) -> i32;
    pub fn mv_batch_stats(ctx: *mut mv_ctx, batches: *mut u64, fallbacks: *mut u64) -> i32;
    pub fn mv_batch_counters(ctx: *mut mv_ctx, out: *mut u64) -> i32;
    pub fn mv_batch_routes(ctx: *mut mv_ctx, out: *mut u64) -> i32;
    pub fn mv_set_batch_groups(ctx: *mut mv_ctx, groups: u32) -> i32;
    pub fn mv_set_stage_timing(ctx: *mut mv_ctx, enable: i32) -> i32;
    pub fn mv_stage_times(ctx: *mut mv_ctx, ms: *mut f64, calls: *mut u64, reset: i32) -> i32;
    pub fn mv_selftest(ctx: *mut mv_ctx, op: i32, input: *const u32, n: u32, out: *mut u32) -> i32;
    pub fn mv_set_option(ctx: *mut mv_ctx, name: *const c_char, value: i64) -> i32;
    pub fn mv_get_option(ctx: *mut mv_ctx, name: *const c_char, value: *mut i64) -> i32;
}
