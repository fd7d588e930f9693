"""mysticeti_amd — MI355X (gfx950) StatementBlock verification engine.

Python host binding of libmysti_verify.so (C ABI: include/mysti_verify.h). The
GPU path is the only path: importing works without a GPU, but every compute call
goes through the HIP library and raises if it (or a device) is missing — there is
no CPU fallback.

Reference interfaces mirrored (hrubaanna/mysticeti @ 2025-02-04):
  Engine.verify_blocks     NetworkSyncer::process_blocks' per-block StatementBlock::verify
                           (net_sync.rs:331-375, types.rs:315-376)
  Engine.ed25519_verify    PublicKey::verify_block -> VerificationKey::verify (crypto.rs:174-189)
  Engine.ed25519_sign      Signer::sign_block (crypto.rs:199-223)
  Engine.blake2b256        BlockHasher (crypto.rs:34)
  Engine.crc32             crc32fast::hash as the WAL uses it (wal.rs:173-177, :250)
  Engine.wal_verify        WalReader::iter_until / WalIterator over try_read (wal.rs:226-346)
  Engine.wal_iter_until    the same as the reference's iterator: (pos, (tag, bytes)), raising
                           where the reference panics
  wal_layout               WalWriter::writev positions (wal.rs:150-188)
  crypto.*                 thin reference-named wrappers (BlockDigest, PublicKey, Signer, ...)
"""
from __future__ import annotations

import contextlib
import ctypes
import os
from typing import Iterable, List, Optional, Sequence, Tuple

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# MV_LIB selects an experiment build (python -m mysticeti_amd.build --variant NAME -D...)
LIB_PATH = os.environ.get("MV_LIB") or os.path.join(_HERE, "libmysti_verify.so")

MV_OK = 0
SIG_OK, SIG_INVALID, SIG_MALFORMED_KEY = 0, 1, 2
BLOCK_STATUS = [
    "OK", "PARSE_ERROR", "DIGEST_MISMATCH", "EPOCH_MISMATCH", "UNKNOWN_AUTHOR", "GENESIS", "SIG_INVALID",
    "INCLUDE_UNKNOWN_AUTHORITY", "INCLUDE_ROUND", "VOTE_RANGE", "THRESHOLD_CLOCK", "VOTE_RANGE_TOO_LONG",
    "VOTE_RANGE_END_TOO_LARGE",
]
(BLOCK_OK, BLOCK_PARSE_ERROR, BLOCK_DIGEST_MISMATCH, BLOCK_EPOCH_MISMATCH, BLOCK_UNKNOWN_AUTHOR,
 BLOCK_GENESIS, BLOCK_SIG_INVALID, BLOCK_INCLUDE_UNKNOWN_AUTHORITY, BLOCK_INCLUDE_ROUND,
 BLOCK_VOTE_RANGE, BLOCK_THRESHOLD_CLOCK, BLOCK_VOTE_RANGE_TOO_LONG, BLOCK_VOTE_RANGE_END_TOO_LARGE) = range(13)

EXPORTS = [
    "mv_create", "mv_destroy", "mv_last_error", "mv_version", "mv_set_committee", "mv_blake2b256",
    "mv_ed25519_verify", "mv_ed25519_sign", "mv_verify_blocks", "mv_dev_ed25519_verify",
    "mv_dev_ed25519_sign", "mv_selftest", "mv_block_preimage", "mv_dev_ed25519_verify_batch", "mv_batch_stats",
    "mv_set_stage_timing", "mv_stage_times", "mv_dev_verify_blocks", "mv_batch_counters", "mv_batch_routes", "mv_set_batch_groups",
    "mv_queue_stats", "mv_shard_plan", "mv_crc32", "mv_wal_verify", "mv_wal_layout", "mv_dev_wal_verify",
    "mv_frame_blocks",
    "mv_dev_crc32", "mv_host_alloc", "mv_host_free", "mv_online_stats", "mv_set_option", "mv_get_option",
]
WAL_OK, WAL_CRC_MISMATCH, WAL_NONZERO_CRC_LEN0, WAL_BAD_LENGTH = range(4)
WAL_MAP_BITS, WAL_MAP_BITS_TEST = 24, 16  # wal.rs:95-103
# batch path stages, the block pipeline's, the WAL replay's (mv_stage_times order, MV_NSTAGES)
STAGES = ["prep", "sort", "bucket", "reduce", "final", "fallback", "parse", "hash", "verify", "verdict", "wal_walk",
          "wal_crc"]
FLAG_NO_BATCH, FLAG_NO_COMB, FLAG_HOST_PARSE, FLAG_NO_ONLINE = 1, 2, 4, 8
BATCH_MIN = 4096


class MvError(RuntimeError):
    pass


class _Config(ctypes.Structure):
    _fields_ = [("device_mask", ctypes.c_uint32), ("max_batch", ctypes.c_uint32), ("flags", ctypes.c_uint32),
                ("shards_per_device", ctypes.c_uint32)]


_lib = None


def load_library(path: str = LIB_PATH):
    """Load libmysti_verify.so (in-tree). Raises if it has not been built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise MvError(f"{path} missing: build it with `python -m mysticeti_amd.build` (no CPU fallback exists)")
    lib = ctypes.CDLL(path)
    vp, u32, u64 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64
    lib.mv_create.argtypes = [ctypes.POINTER(_Config), ctypes.POINTER(vp)]
    lib.mv_destroy.argtypes = [vp]
    lib.mv_destroy.restype = None
    lib.mv_last_error.argtypes = [vp]
    lib.mv_last_error.restype = ctypes.c_char_p
    lib.mv_version.restype = ctypes.c_char_p
    lib.mv_set_committee.argtypes = [vp, vp, vp, u32, u64, vp]
    lib.mv_blake2b256.argtypes = [vp, vp, vp, vp, u32, vp]
    lib.mv_ed25519_verify.argtypes = [vp, vp, vp, vp, vp, u32, vp]
    lib.mv_ed25519_sign.argtypes = [vp, vp, vp, u32, vp, vp]
    lib.mv_verify_blocks.argtypes = [vp, vp, vp, vp, u32, vp, vp, vp]
    lib.mv_dev_ed25519_verify.argtypes = [vp, ctypes.c_int, vp, vp, vp, u32, vp, vp]
    lib.mv_dev_ed25519_verify_batch.argtypes = [vp, ctypes.c_int, vp, vp, vp, vp, u32, vp, vp, vp]
    lib.mv_batch_stats.argtypes = [vp, vp, vp]
    lib.mv_batch_counters.argtypes = [vp, vp]
    lib.mv_batch_routes.argtypes = [vp, vp]
    lib.mv_set_batch_groups.argtypes = [vp, u32]
    lib.mv_queue_stats.argtypes = [vp, vp, vp]
    lib.mv_online_stats.argtypes = [vp, vp, vp]
    lib.mv_shard_plan.argtypes = [vp, u64, u32, vp]
    lib.mv_set_stage_timing.argtypes = [vp, ctypes.c_int]
    lib.mv_stage_times.argtypes = [vp, vp, vp, ctypes.c_int]
    lib.mv_dev_verify_blocks.argtypes = [vp, ctypes.c_int, vp, u64, vp, vp, u32, vp, vp, vp, vp]
    lib.mv_dev_ed25519_sign.argtypes = [vp, ctypes.c_int, vp, vp, u32, vp, vp, vp]
    lib.mv_selftest.argtypes = [vp, ctypes.c_int, vp, u32, vp]
    lib.mv_block_preimage.argtypes = [vp, u64, vp, u64]
    lib.mv_block_preimage.restype = ctypes.c_int64
    lib.mv_crc32.argtypes = [vp, vp, vp, vp, u32, vp]
    lib.mv_wal_verify.argtypes = [vp, vp, u64, u64, u32, vp, vp, vp, vp, u64, vp]
    lib.mv_wal_layout.argtypes = [vp, u64, u32, u64, vp]
    lib.mv_wal_layout.restype = u64
    lib.mv_frame_blocks.argtypes = [vp, u64, vp, vp, u64, vp]
    lib.mv_frame_blocks.restype = ctypes.c_int64
    lib.mv_dev_wal_verify.argtypes = [vp, ctypes.c_int, vp, u64, u64, u32, vp, vp, vp, vp, u64, vp, vp]
    lib.mv_dev_crc32.argtypes = [vp, ctypes.c_int, vp, vp, vp, u32, vp, vp]
    lib.mv_host_alloc.argtypes = [vp, u64, ctypes.POINTER(vp)]
    lib.mv_host_free.argtypes = [vp, vp]
    lib.mv_host_free.restype = None
    lib.mv_set_option.argtypes = [vp, ctypes.c_char_p, ctypes.c_int64]
    lib.mv_get_option.argtypes = [vp, ctypes.c_char_p, ctypes.POINTER(ctypes.c_int64)]
    for name in EXPORTS:
        getattr(lib, name).restype = getattr(lib, name).restype or ctypes.c_int32
    _lib = lib
    return lib


def _p(a: Optional[np.ndarray]):
    return None if a is None else ctypes.c_void_p(a.ctypes.data)


def _u8(a, shape_tail: int) -> np.ndarray:
    a = np.ascontiguousarray(np.asarray(a, dtype=np.uint8))
    return a.reshape(-1, shape_tail)


class Engine:
    """One mv_ctx: the devices it shards over, their streams and buffers."""

    def __init__(self, devices: Sequence[int] = (0,), max_batch: int = 0, batch: bool = True, comb: bool = True,
                 host_parse: bool = False, shards_per_device: int = 1, online: bool = True):
        """batch=False sets MV_FLAG_NO_BATCH: host-buffer verifies check every signature alone.
        comb=False sets MV_FLAG_NO_COMB: committee keys go through the per-signature ladder,
        not the per-key comb tables. host_parse=True sets MV_FLAG_HOST_PARSE: verify_blocks
        parses the bincode on the host instead of on the GPU. shards_per_device > 1 makes
        that many logical shards per device (host calls shard across them as across GPUs).
        online=False sets MV_FLAG_NO_ONLINE: small verify_blocks calls skip the resident online
        service and go through the submission queue."""
        self.lib = load_library()
        mask = 0
        for d in devices:
            mask |= 1 << int(d)
        flags = (0 if batch else FLAG_NO_BATCH) | (0 if comb else FLAG_NO_COMB) | (FLAG_HOST_PARSE if host_parse else 0) \
            | (0 if online else FLAG_NO_ONLINE)
        cfg = _Config(mask, max_batch, flags, shards_per_device)
        h = ctypes.c_void_p()
        rc = self.lib.mv_create(ctypes.byref(cfg), ctypes.byref(h))
        if rc != MV_OK:
            raise MvError(f"mv_create failed ({rc}): no usable gfx950 device")
        self.ctx = h
        self.devices = list(devices)

    def close(self):
        if getattr(self, "ctx", None):
            for ptr in getattr(self, "_pinned", {}).values():
                self.lib.mv_host_free(self.ctx, ptr)
            self._pinned = {}
            self.lib.mv_destroy(self.ctx)
            self.ctx = None

    def host_empty(self, shape, dtype=np.uint8) -> np.ndarray:
        """A numpy array in page-locked host memory (mv_host_alloc), valid until close(): verify
        inputs held in such arrays are streamed to the GPU beside the verification."""
        nbytes = int(np.prod(shape)) * np.dtype(dtype).itemsize
        ptr = ctypes.c_void_p()
        self._check(self.lib.mv_host_alloc(self.ctx, max(nbytes, 1), ctypes.byref(ptr)), "mv_host_alloc")
        if not hasattr(self, "_pinned"):
            self._pinned = {}
        self._pinned[ptr.value] = ptr
        raw = (ctypes.c_uint8 * max(nbytes, 1)).from_address(ptr.value)
        return np.frombuffer(raw, dtype=np.uint8, count=nbytes).view(dtype).reshape(shape)

    def host_free(self, arr: np.ndarray):
        """Releases an array from host_empty (it must not be used afterwards)."""
        ptr = getattr(self, "_pinned", {}).pop(arr.__array_interface__["data"][0], None)
        if ptr is not None:
            self.lib.mv_host_free(self.ctx, ptr)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def _check(self, rc: int, what: str):
        if rc != MV_OK:
            raise MvError(f"{what} failed ({rc}): {self.lib.mv_last_error(self.ctx).decode()}")

    # ---- runtime switches (mv_set_option: the environment is read once, at mv_create) ----
    def set_option(self, name: str, value: int):
        self._check(self.lib.mv_set_option(self.ctx, name.encode(), int(value)), f"mv_set_option({name})")

    def get_option(self, name: str) -> int:
        v = ctypes.c_int64()
        self._check(self.lib.mv_get_option(self.ctx, name.encode(), ctypes.byref(v)), f"mv_get_option({name})")
        return v.value

    @contextlib.contextmanager
    def option(self, name: str, value: int):
        """Sets a runtime switch for the duration of a with-block (then restores it)."""
        old = self.get_option(name)
        self.set_option(name, value)
        try:
            yield self
        finally:
            self.set_option(name, old)

    # ---- committee ----
    def set_committee(self, pks, stakes, epoch: int = 0) -> np.ndarray:
        pks = _u8(pks, 32)
        stakes = np.ascontiguousarray(np.asarray(stakes, dtype=np.uint64))
        ok = np.zeros(pks.shape[0], dtype=np.uint8)
        self._check(self.lib.mv_set_committee(self.ctx, _p(pks), _p(stakes), pks.shape[0], epoch, _p(ok)),
                    "mv_set_committee")
        return ok

    # ---- hashes ----
    def blake2b256(self, items: Sequence[bytes]) -> List[bytes]:
        n = len(items)
        lens = np.array([len(x) for x in items], dtype=np.uint64)
        offs = np.zeros(n, dtype=np.uint64)
        if n > 1:
            offs[1:] = np.cumsum(lens)[:-1]
        buf = np.frombuffer(b"".join(items) + b"\0", dtype=np.uint8)
        out = np.zeros((n, 32), dtype=np.uint8)
        self._check(self.lib.mv_blake2b256(self.ctx, _p(buf), _p(offs), _p(lens), n, _p(out)), "mv_blake2b256")
        return [bytes(r) for r in out]

    # ---- signatures ----
    def ed25519_verify(self, msg, sig, pk=None, key_idx=None) -> np.ndarray:
        msg, sig = _u8(msg, 32), _u8(sig, 64)
        n = msg.shape[0]
        pk_a = _u8(pk, 32) if pk is not None else None
        ki = np.ascontiguousarray(np.asarray(key_idx, dtype=np.uint32)) if key_idx is not None else None
        st = np.zeros(n, dtype=np.uint8)
        self._check(self.lib.mv_ed25519_verify(self.ctx, _p(msg), _p(sig), _p(pk_a), _p(ki), n, _p(st)),
                    "mv_ed25519_verify")
        return st

    def ed25519_sign(self, seed, msg) -> Tuple[np.ndarray, np.ndarray]:
        seed, msg = _u8(seed, 32), _u8(msg, 32)
        n = seed.shape[0]
        pk = np.zeros((n, 32), dtype=np.uint8)
        sig = np.zeros((n, 64), dtype=np.uint8)
        self._check(self.lib.mv_ed25519_sign(self.ctx, _p(seed), _p(msg), n, _p(pk), _p(sig)), "mv_ed25519_sign")
        return pk, sig

    # ---- blocks ----
    def verify_blocks(self, blocks: Sequence[bytes]):
        """StatementBlock::verify for each bincode Data<StatementBlock>: (status, msg_digest, block_digest)."""
        n = len(blocks)
        lens = np.array([len(b) for b in blocks], dtype=np.uint64)
        offs = np.zeros(n, dtype=np.uint64)
        if n > 1:
            offs[1:] = np.cumsum(lens)[:-1]
        buf = np.frombuffer(b"".join(blocks) + b"\0", dtype=np.uint8)
        return self.verify_blocks_packed(buf, offs, lens)

    def verify_blocks_packed(self, buf: np.ndarray, offs: np.ndarray, lens: np.ndarray):
        n = offs.shape[0]
        buf = np.ascontiguousarray(buf, dtype=np.uint8)
        offs = np.ascontiguousarray(offs, dtype=np.uint64)
        lens = np.ascontiguousarray(lens, dtype=np.uint64)
        st = np.zeros(n, dtype=np.uint8)
        md = np.zeros((n, 32), dtype=np.uint8)
        bd = np.zeros((n, 32), dtype=np.uint8)
        self._check(self.lib.mv_verify_blocks(self.ctx, _p(buf), _p(offs), _p(lens), n, _p(st), _p(md), _p(bd)),
                    "mv_verify_blocks")
        return st, md, bd

    def verify_frames(self, buf):
        """Blocks of received NetworkMessage frames (network.rs:400-447) verified in place:
        mv_frame_blocks lists them, mv_verify_blocks checks them on the same buffer. Returns
        (status, msg_digest, block_digest, consumed bytes of complete frames)."""
        buf = np.ascontiguousarray(np.frombuffer(buf, dtype=np.uint8) if isinstance(buf, (bytes, bytearray)) else buf,
                                   dtype=np.uint8)
        offs, lens, consumed = frame_blocks(buf)
        st, md, bd = self.verify_blocks_packed(buf, offs, lens)
        return st, md, bd, consumed

    # ---- device-resident (torch tensors on the device) ----
    def dev_verify(self, device: int, d_msg, d_sig, d_pk, d_status, stream_handle: int = 0):
        n = d_msg.shape[0]
        self._check(self.lib.mv_dev_ed25519_verify(self.ctx, device, ctypes.c_void_p(d_msg.data_ptr()),
                                                   ctypes.c_void_p(d_sig.data_ptr()), ctypes.c_void_p(d_pk.data_ptr()),
                                                   n, ctypes.c_void_p(d_status.data_ptr()),
                                                   ctypes.c_void_p(stream_handle or None)),
                    "mv_dev_ed25519_verify")

    def dev_verify_batch(self, device: int, d_msg, d_sig, d_pk, d_status, d_batch_ok=None, stream_handle: int = 0,
                         d_key_idx=None):
        """Batch path (one combined equation, exact fallback) on device tensors; enqueue only."""
        n = d_msg.shape[0]
        vp = ctypes.c_void_p
        self._check(self.lib.mv_dev_ed25519_verify_batch(
            self.ctx, device, vp(d_msg.data_ptr()), vp(d_sig.data_ptr()), vp(d_pk.data_ptr()),
            vp(d_key_idx.data_ptr()) if d_key_idx is not None else None, n, vp(d_status.data_ptr()),
            vp(d_batch_ok.data_ptr()) if d_batch_ok is not None else None, vp(stream_handle or None)),
            "mv_dev_ed25519_verify_batch")

    def batch_stats(self) -> Tuple[int, int]:
        """(batches tried, batches that fell back to per-signature verification) on the host path."""
        b, f = ctypes.c_uint64(), ctypes.c_uint64()
        self._check(self.lib.mv_batch_stats(self.ctx, ctypes.byref(b), ctypes.byref(f)), "mv_batch_stats")
        return b.value, f.value

    def batch_counters(self) -> Tuple[int, int, int, int]:
        """(batches, batches with a failed equation, sub-batch equations, failed sub-batch equations)."""
        out = np.zeros(4, dtype=np.uint64)
        self._check(self.lib.mv_batch_counters(self.ctx, _p(out)), "mv_batch_counters")
        return tuple(int(x) for x in out)

    def batch_routes(self) -> Tuple[int, int, int]:
        """(batches checked by a combined equation, batches verified signature by signature
        because failures were dense, dense failures seen)."""
        out = np.zeros(3, dtype=np.uint64)
        self._check(self.lib.mv_batch_routes(self.ctx, _p(out)), "mv_batch_routes")
        return tuple(int(x) for x in out)

    def set_batch_groups(self, groups: int):
        """Sub-batch equations per batch: 0 = adaptive (default), 1..16 fixed."""
        self._check(self.lib.mv_set_batch_groups(self.ctx, int(groups)), "mv_set_batch_groups")

    def queue_stats(self) -> Tuple[int, int]:
        """(mv_verify_blocks calls, device passes that served them)."""
        c, p = ctypes.c_uint64(), ctypes.c_uint64()
        self._check(self.lib.mv_queue_stats(self.ctx, ctypes.byref(c), ctypes.byref(p)), "mv_queue_stats")
        return c.value, p.value

    def online_stats(self) -> Tuple[int, int]:
        """(verify_blocks calls served by the resident online service, its kernel launches)."""
        r, l = ctypes.c_uint64(), ctypes.c_uint64()
        self._check(self.lib.mv_online_stats(self.ctx, ctypes.byref(r), ctypes.byref(l)), "mv_online_stats")
        return r.value, l.value

    def set_stage_timing(self, enable: bool = True):
        self._check(self.lib.mv_set_stage_timing(self.ctx, 1 if enable else 0), "mv_set_stage_timing")

    def stage_times(self, reset: bool = False):
        """({stage: summed device ms}, {stage: calls measured}) since the last reset."""
        ms = np.zeros(len(STAGES), dtype=np.float64)
        calls = np.zeros(len(STAGES), dtype=np.uint64)
        self._check(self.lib.mv_stage_times(self.ctx, _p(ms), _p(calls), 1 if reset else 0), "mv_stage_times")
        return dict(zip(STAGES, ms.tolist())), dict(zip(STAGES, (int(c) for c in calls)))

    def dev_verify_blocks(self, device: int, d_buf, buf_bytes: int, d_off, d_len, d_status, d_md=None, d_bd=None,
                          stream_handle: int = 0):
        """StatementBlock::verify on HBM-resident bincode (torch uint8 buffer, int64 offsets and
        lengths); parse, digests, signatures and checks on the GPU. Enqueue only."""
        n = d_off.shape[0]
        vp = ctypes.c_void_p
        self._check(self.lib.mv_dev_verify_blocks(
            self.ctx, device, vp(d_buf.data_ptr()), int(buf_bytes), vp(d_off.data_ptr()), vp(d_len.data_ptr()), n,
            vp(d_status.data_ptr()), vp(d_md.data_ptr()) if d_md is not None else None,
            vp(d_bd.data_ptr()) if d_bd is not None else None, vp(stream_handle or None)), "mv_dev_verify_blocks")

    def dev_sign(self, device: int, d_seed, d_msg, d_pk, d_sig, stream_handle: int = 0):
        n = d_seed.shape[0]
        self._check(self.lib.mv_dev_ed25519_sign(self.ctx, device, ctypes.c_void_p(d_seed.data_ptr()),
                                                 ctypes.c_void_p(d_msg.data_ptr()), n,
                                                 ctypes.c_void_p(d_pk.data_ptr()), ctypes.c_void_p(d_sig.data_ptr()),
                                                 ctypes.c_void_p(stream_handle or None)),
                    "mv_dev_ed25519_sign")

    # ---- WAL replay (wal.rs) ----
    def crc32(self, items: Sequence[bytes]) -> np.ndarray:
        """crc32fast::hash of every item (uint32 array)."""
        items = [bytes(x) for x in items]
        lens = np.array([len(x) for x in items], dtype=np.uint64)
        offs = np.zeros(len(items), dtype=np.uint64)
        if len(items) > 1:
            offs[1:] = np.cumsum(lens)[:-1]
        buf = np.frombuffer(b"".join(items) + b"\0", dtype=np.uint8)
        return self.crc32_packed(buf, offs, lens)

    def crc32_packed(self, buf: np.ndarray, offs: np.ndarray, lens: np.ndarray) -> np.ndarray:
        buf = np.ascontiguousarray(buf, dtype=np.uint8)
        offs = np.ascontiguousarray(offs, dtype=np.uint64)
        lens = np.ascontiguousarray(lens, dtype=np.uint64)
        n = len(offs)
        out = np.zeros(n, dtype=np.uint32)
        if n:
            self._check(self.lib.mv_crc32(self.ctx, _p(buf), _p(offs), _p(lens), n, _p(out)), "mv_crc32")
        return out

    def wal_verify(self, image, end_pos: Optional[int] = None, map_bits: int = WAL_MAP_BITS,
                   cap: Optional[int] = None):
        """WalReader::iter_until over a WAL image (bytes / uint8 array) up to the writer position
        end_pos (default: its length). Returns (pos, tag, len, status) arrays of the entries in
        iteration order, the last one failing (status != WAL_OK) where the reference panics."""
        img = np.ascontiguousarray(np.frombuffer(image, dtype=np.uint8) if isinstance(image, (bytes, bytearray))
                                   else np.asarray(image, dtype=np.uint8))
        size = img.size
        end = size if end_pos is None else int(end_pos)
        if cap is None:
            cap = size // 16 + 1
        pos = np.zeros(max(cap, 1), dtype=np.uint64)
        tag = np.zeros(max(cap, 1), dtype=np.uint32)
        ln = np.zeros(max(cap, 1), dtype=np.uint32)
        st = np.zeros(max(cap, 1), dtype=np.uint8)
        cnt = ctypes.c_uint64(0)
        self._check(self.lib.mv_wal_verify(self.ctx, _p(img) if size else None, size, end, map_bits, _p(pos),
                                           _p(tag), _p(ln), _p(st), cap, ctypes.byref(cnt)), "mv_wal_verify")
        n = min(cnt.value, cap)
        return pos[:n], tag[:n], ln[:n], st[:n]

    def wal_iter_until(self, image, end_pos: Optional[int] = None, map_bits: int = WAL_MAP_BITS):
        """The reference's iterator (wal.rs:270-346): yields (position, (tag, payload bytes)) and
        raises MvError with the reference's panic message where it would panic."""
        img = bytes(image)
        pos, tag, ln, st = self.wal_verify(img, end_pos, map_bits)
        for p, t, n, s in zip(pos.tolist(), tag.tolist(), ln.tolist(), st.tolist()):
            if s == WAL_CRC_MISMATCH:
                hdr = int.from_bytes(img[p:p + 16].ljust(16, b"\0"), "little")
                full = (hdr >> 64) & 0xFFFFFFFF
                found = int(self.crc32([img[p + 16:p + full].ljust(full - 16, b"\0")])[0])
                raise MvError(f"Crc mismatch, expected {hdr & ((1 << 64) - 1)}, found {found} at position {p}:{full}")
            if s == WAL_NONZERO_CRC_LEN0:
                crc = int.from_bytes(img[p:p + 8].ljust(8, b"\0"), "little")
                raise MvError(f"Non-zero crc at len 0, crc: {crc}, position:{p}")
            if s == WAL_BAD_LENGTH:
                raise MvError(f"entry at position {p} runs outside its map (Bytes::slice out of range)")
            yield p, (t, img[p + 16:p + 16 + n])

    def dev_wal_verify(self, device: int, d_img, size: int, end_pos: int, map_bits: int, d_pos, d_tag, d_len,
                       d_status, cap: int, stream_handle: int = 0) -> int:
        """mv_dev_wal_verify on torch device tensors; returns the entry count."""
        cnt = ctypes.c_uint64(0)
        ptr = lambda t: ctypes.c_void_p(t.data_ptr())
        self._check(self.lib.mv_dev_wal_verify(self.ctx, device, ptr(d_img), size, end_pos, map_bits, ptr(d_pos),
                                               ptr(d_tag), ptr(d_len), ptr(d_status), cap, ctypes.byref(cnt),
                                               ctypes.c_void_p(stream_handle or None)), "mv_dev_wal_verify")
        return cnt.value

    def dev_crc32(self, device: int, d_buf, d_off, d_len, n: int, d_out, stream_handle: int = 0):
        ptr = lambda t: ctypes.c_void_p(t.data_ptr())
        self._check(self.lib.mv_dev_crc32(self.ctx, device, ptr(d_buf), ptr(d_off), ptr(d_len), n, ptr(d_out),
                                          ctypes.c_void_p(stream_handle or None)), "mv_dev_crc32")

    # ---- diagnostics ----
    def selftest(self, op: int, words: np.ndarray) -> np.ndarray:
        w = np.ascontiguousarray(np.asarray(words, dtype=np.uint32)).reshape(-1, 16)
        out = np.zeros_like(w)
        self._check(self.lib.mv_selftest(self.ctx, op, _p(w), w.shape[0], _p(out)), "mv_selftest")
        return out


def block_preimage(bincode: bytes) -> Optional[bytes]:
    """Host-side pre-image of one bincode StatementBlock (None if it does not deserialize)."""
    lib = load_library()
    b = np.frombuffer(bincode + b"\0", dtype=np.uint8)
    n = lib.mv_block_preimage(_p(b), len(bincode), None, 0)
    if n < 0:
        return None
    out = np.zeros(max(n, 1), dtype=np.uint8)
    lib.mv_block_preimage(_p(b), len(bincode), _p(out), n)
    return out[:n].tobytes()


def shard_plan(weights, parts: int) -> List[int]:
    """Host-only: the contiguous shard cuts the multi-device paths use (balanced by weight)."""
    lib = load_library()
    w = np.ascontiguousarray(np.asarray(weights, dtype=np.uint64))
    cut = np.zeros(parts + 1, dtype=np.uint64)
    rc = lib.mv_shard_plan(_p(w) if w.size else None, w.size, parts, _p(cut))
    if rc != MV_OK:
        raise MvError(f"mv_shard_plan failed ({rc})")
    return [int(c) for c in cut]


def wal_layout(payload_lens, map_bits: int = WAL_MAP_BITS, start: int = 0):
    """Host-only: WalWriter::writev positions of entries with these payload lengths, and the
    writer position after them."""
    lib = load_library()
    pl = np.ascontiguousarray(np.asarray(payload_lens, dtype=np.uint64))
    pos = np.zeros(max(pl.size, 1), dtype=np.uint64)
    end = lib.mv_wal_layout(_p(pl) if pl.size else None, pl.size, map_bits, start, _p(pos))
    return pos[:pl.size], int(end)


def frame_blocks(buf) -> Tuple[np.ndarray, np.ndarray, int]:
    """Host-only: (offsets, lengths) of the Data<StatementBlock> byte strings inside received
    NetworkMessage frames (mv_frame_blocks, network.rs:400-447), and the bytes of the complete
    frames. Raises MvError where the reference would drop the connection."""
    lib = load_library()
    b = np.ascontiguousarray(np.frombuffer(buf, dtype=np.uint8) if isinstance(buf, (bytes, bytearray)) else buf,
                             dtype=np.uint8)
    consumed = ctypes.c_uint64(0)
    n = lib.mv_frame_blocks(_p(b) if b.size else None, b.size, None, None, 0, ctypes.byref(consumed))
    if n < 0:
        raise MvError("mv_frame_blocks: a malformed frame stream (the reference drops the connection)")
    offs = np.zeros(max(n, 1), dtype=np.uint64)
    lens = np.zeros(max(n, 1), dtype=np.uint64)
    lib.mv_frame_blocks(_p(b) if b.size else None, b.size, _p(offs), _p(lens), n, ctypes.byref(consumed))
    return offs[:n], lens[:n], int(consumed.value)


def version() -> str:
    return load_library().mv_version().decode()
