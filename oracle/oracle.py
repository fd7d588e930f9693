"""ORACLE / TEST INFRASTRUCTURE ONLY: ctypes binding of the C restatement.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this,
as the checker. See oracle/oracle.h for what it restates (file:line).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "libmv_oracle.so")
_lib = None

SIG_OK, SIG_INVALID, SIG_MALFORMED_KEY = 0, 1, 2
(BLOCK_OK, BLOCK_PARSE_ERROR, BLOCK_DIGEST_MISMATCH, BLOCK_EPOCH_MISMATCH, BLOCK_UNKNOWN_AUTHOR,
 BLOCK_GENESIS, BLOCK_SIG_INVALID, BLOCK_INCLUDE_UNKNOWN_AUTHORITY, BLOCK_INCLUDE_ROUND,
 BLOCK_VOTE_RANGE, BLOCK_THRESHOLD_CLOCK, BLOCK_VOTE_RANGE_TOO_LONG, BLOCK_VOTE_RANGE_END_TOO_LARGE) = range(13)


def build(force: bool = False, archflags: str | None = None) -> str:
    """Compile oracle/build/libmv_oracle.so with make (gcc)."""
    cmd = ["make", "-C", _HERE, "-s"]
    if archflags is not None:
        cmd.append(f"ARCHFLAGS={archflags}")
    if force:
        subprocess.run(["make", "-C", _HERE, "-s", "clean"], check=True)
    subprocess.run(cmd, check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        _lib = ctypes.CDLL(_LIB_PATH)
        u8p = ctypes.c_void_p
        _lib.orc_blake2b256.argtypes = [u8p, ctypes.c_size_t, u8p]
        _lib.orc_sha512.argtypes = [u8p, ctypes.c_size_t, u8p]
        _lib.orc_ed25519_verify.argtypes = [u8p, u8p, u8p, ctypes.c_size_t]
        _lib.orc_ed25519_verify.restype = ctypes.c_int
        _lib.orc_ed25519_pubkey.argtypes = [u8p, u8p]
        _lib.orc_ed25519_sign.argtypes = [u8p, u8p, ctypes.c_size_t, u8p]
        _lib.orc_point_decodes.argtypes = [u8p]
        _lib.orc_point_decodes.restype = ctypes.c_int
        _lib.orc_scalar_reduce_wide.argtypes = [u8p, u8p]
        _lib.orc_ed25519_verify_batch.argtypes = [u8p, u8p, u8p, ctypes.c_size_t, u8p, ctypes.c_int]
        _lib.orc_ed25519_sign_batch.argtypes = [u8p, u8p, ctypes.c_size_t, u8p, u8p, ctypes.c_int]
        _lib.orc_block_preimage.argtypes = [u8p, ctypes.c_size_t, u8p, ctypes.c_size_t]
        _lib.orc_block_preimage.restype = ctypes.c_long
        _lib.orc_block_verify.argtypes = [u8p, ctypes.c_size_t, u8p, u8p, ctypes.c_uint32, ctypes.c_uint64, u8p,
                                          u8p]
        _lib.orc_block_verify.restype = ctypes.c_int
        _lib.orc_block_verify_batch.argtypes = [u8p, u8p, u8p, ctypes.c_size_t, u8p, u8p, ctypes.c_uint32,
                                                ctypes.c_uint64, u8p, u8p, u8p, ctypes.c_int]
        _lib.orc_committee_new.argtypes = [u8p, u8p, ctypes.c_uint32, ctypes.c_uint64]
        _lib.orc_committee_new.restype = ctypes.c_void_p
        _lib.orc_committee_free.argtypes = [u8p]
        _lib.orc_block_verify_batch_c.argtypes = [u8p, u8p, u8p, u8p, ctypes.c_size_t, u8p, u8p, u8p, ctypes.c_int]
        _lib.orc_crc32.argtypes = [u8p, ctypes.c_size_t]
        _lib.orc_crc32.restype = ctypes.c_uint32
        _lib.orc_crc32_table.argtypes = [u8p, ctypes.c_size_t]
        _lib.orc_crc32_table.restype = ctypes.c_uint32
        _lib.orc_crc32_batch.argtypes = [u8p, u8p, u8p, ctypes.c_size_t, u8p]
        _lib.orc_wal_layout.argtypes = [u8p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint64, u8p]
        _lib.orc_wal_layout.restype = ctypes.c_uint64
        _lib.orc_wal_iter.argtypes = [u8p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32, u8p, u8p, u8p, u8p,
                                      ctypes.c_uint64]
        _lib.orc_wal_iter.restype = ctypes.c_uint64
    return _lib


def _buf(b: bytes):
    return ctypes.c_char_p(b) if b else None


def _ptr(a: np.ndarray):
    return ctypes.c_void_p(a.ctypes.data) if a is not None else None


def blake2b256(data: bytes) -> bytes:
    out = ctypes.create_string_buffer(32)
    lib().orc_blake2b256(_buf(data), len(data), out)
    return out.raw


def sha512(data: bytes) -> bytes:
    out = ctypes.create_string_buffer(64)
    lib().orc_sha512(_buf(data), len(data), out)
    return out.raw


def verify(pk: bytes, sig: bytes, msg: bytes) -> int:
    return lib().orc_ed25519_verify(_buf(pk), _buf(sig), _buf(msg), len(msg))


def public_key(seed: bytes) -> bytes:
    out = ctypes.create_string_buffer(32)
    lib().orc_ed25519_pubkey(_buf(seed), out)
    return out.raw


def sign(seed: bytes, msg: bytes) -> bytes:
    out = ctypes.create_string_buffer(64)
    lib().orc_ed25519_sign(_buf(seed), _buf(msg), len(msg), out)
    return out.raw


def point_decodes(enc: bytes) -> bool:
    return bool(lib().orc_point_decodes(_buf(enc)))


def scalar_reduce_wide(b64: bytes) -> bytes:
    out = ctypes.create_string_buffer(32)
    lib().orc_scalar_reduce_wide(_buf(b64), out)
    return out.raw


def verify_batch(pk: np.ndarray, sig: np.ndarray, msg: np.ndarray, threads: int = 0) -> np.ndarray:
    n = pk.shape[0]
    pk, sig, msg = (np.ascontiguousarray(x, dtype=np.uint8) for x in (pk, sig, msg))
    status = np.zeros(n, dtype=np.uint8)
    lib().orc_ed25519_verify_batch(_ptr(pk), _ptr(sig), _ptr(msg), n, _ptr(status), threads)
    return status


def sign_batch(seed: np.ndarray, msg: np.ndarray, threads: int = 0):
    n = seed.shape[0]
    seed, msg = (np.ascontiguousarray(x, dtype=np.uint8) for x in (seed, msg))
    pk = np.zeros((n, 32), dtype=np.uint8)
    sig = np.zeros((n, 64), dtype=np.uint8)
    lib().orc_ed25519_sign_batch(_ptr(seed), _ptr(msg), n, _ptr(pk), _ptr(sig), threads)
    return pk, sig


def block_preimage(bincode: bytes) -> bytes | None:
    n = lib().orc_block_preimage(_buf(bincode), len(bincode), None, 0)
    if n < 0:
        return None
    out = ctypes.create_string_buffer(max(n, 1))
    lib().orc_block_preimage(_buf(bincode), len(bincode), out, n)
    return out.raw[:n]


def block_verify(bincode: bytes, pks: np.ndarray, stakes: np.ndarray, epoch: int):
    md = ctypes.create_string_buffer(32)
    bd = ctypes.create_string_buffer(32)
    pks = np.ascontiguousarray(pks, dtype=np.uint8)
    stakes = np.ascontiguousarray(stakes, dtype=np.uint64)
    st = lib().orc_block_verify(_buf(bincode), len(bincode), _ptr(pks), _ptr(stakes), pks.shape[0], epoch, md, bd)
    return st, md.raw, bd.raw


def block_verify_batch(buf: np.ndarray, off: np.ndarray, lens: np.ndarray, pks: np.ndarray, stakes: np.ndarray,
                       epoch: int, threads: int = 0, decoded_committee: bool = False):
    """StatementBlock::verify of every block; decoded_committee: through orc_committee (keys
    decoded once, as the reference's Committee holds them) instead of a decode per verify."""
    n = off.shape[0]
    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    off = np.ascontiguousarray(off, dtype=np.uint64)
    lens = np.ascontiguousarray(lens, dtype=np.uint64)
    pks = np.ascontiguousarray(pks, dtype=np.uint8)
    stakes = np.ascontiguousarray(stakes, dtype=np.uint64)
    status = np.zeros(n, dtype=np.uint8)
    md = np.zeros((n, 32), dtype=np.uint8)
    bd = np.zeros((n, 32), dtype=np.uint8)
    if decoded_committee:
        c = lib().orc_committee_new(_ptr(pks), _ptr(stakes), pks.shape[0], epoch)
        try:
            lib().orc_block_verify_batch_c(c, _ptr(buf), _ptr(off), _ptr(lens), n, _ptr(status), _ptr(md), _ptr(bd),
                                           threads)
        finally:
            lib().orc_committee_free(c)
        return status, md, bd
    lib().orc_block_verify_batch(_ptr(buf), _ptr(off), _ptr(lens), n, _ptr(pks), _ptr(stakes), pks.shape[0], epoch,
                                 _ptr(status), _ptr(md), _ptr(bd), threads)
    return status, md, bd


WAL_OK, WAL_CRC_MISMATCH, WAL_NONZERO_CRC_LEN0, WAL_BAD_LENGTH = range(4)


def crc32(data: bytes) -> int:
    """crc32fast::hash (oracle/wal.c)."""
    b = np.frombuffer(bytes(data) or b"\0", dtype=np.uint8)
    return int(lib().orc_crc32(_ptr(b), len(data)))


def crc32_table(data: bytes) -> int:
    """The byte-at-a-time table form (oracle/wal.c), to cross-check the folded one."""
    b = np.frombuffer(bytes(data) or b"\0", dtype=np.uint8)
    return int(lib().orc_crc32_table(_ptr(b), len(data)))


def crc32_batch(buf: np.ndarray, off: np.ndarray, lens: np.ndarray) -> np.ndarray:
    out = np.zeros(len(off), dtype=np.uint32)
    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    off = np.ascontiguousarray(off, dtype=np.uint64)
    lens = np.ascontiguousarray(lens, dtype=np.uint64)
    lib().orc_crc32_batch(_ptr(buf), _ptr(off), _ptr(lens), len(off), _ptr(out))
    return out


def wal_layout(payload_len, map_bits: int, start: int = 0):
    """WalWriter::writev positions (oracle/wal.c) -> (positions, writer position after)."""
    pl = np.ascontiguousarray(payload_len, dtype=np.uint64)
    pos = np.zeros(max(len(pl), 1), dtype=np.uint64)
    end = lib().orc_wal_layout(_ptr(pl), len(pl), map_bits, start, _ptr(pos))
    return pos[:len(pl)], int(end)


def wal_iter(img: np.ndarray, end_pos: int, map_bits: int, cap: int | None = None):
    """WalReader::iter_until (oracle/wal.c) -> (pos, tag, len, status) arrays of the entries read,
    the last one failing if the reference would panic there."""
    img = np.ascontiguousarray(img, dtype=np.uint8)
    if cap is None:
        cap = len(img) // 16 + 2
    pos = np.zeros(cap, dtype=np.uint64)
    tag = np.zeros(cap, dtype=np.uint32)
    ln = np.zeros(cap, dtype=np.uint32)
    st = np.zeros(cap, dtype=np.uint8)
    n = lib().orc_wal_iter(_ptr(img) if len(img) else None, len(img), end_pos, map_bits, _ptr(pos), _ptr(tag),
                           _ptr(ln), _ptr(st), cap)
    n = min(int(n), cap)
    return pos[:n], tag[:n], ln[:n], st[:n]
