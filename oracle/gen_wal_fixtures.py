"""ORACLE / TEST INFRASTRUCTURE ONLY: writes tests/golden/wal.json.

    python oracle/gen_wal_fixtures.py

crc32 vectors come from zlib.crc32 (CRC-32/ISO-HDLC, the function crc32fast::hash computes).
WAL scenarios are built with oracle/wal.py's WalWriter and their expected iteration is computed
by `iterate` below, a line-by-line Python restatement of WalIterator::next / try_position /
WalReader::try_read (mysticeti-core/src/wal.rs:226-346), cross-checked against the C
restatement (oracle/wal.c) before anything is written. The first two scenarios are the
reference's own tests (wal.rs:380-446 test_wal, wal.rs:448-473
test_wal_iterator_over_map_boundary) with the positions, tags and payloads they assert.
Images are stored as a recipe (entries, corruptions) plus their SHA-256, not as bytes.
"""
from __future__ import annotations

import hashlib
import json
import os
import struct
import sys
import zlib

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import oracle as O  # noqa: E402
import wal as W  # noqa: E402

OUT = os.path.join(HERE, "..", "tests", "golden", "wal.json")


def pattern(n: int, seed: int) -> bytes:
    """Deterministic payload bytes (no RNG-version dependence)."""
    i = np.arange(n, dtype=np.uint64) + np.uint64(seed) * np.uint64(0x9E3779B1)
    return (((i * np.uint64(2654435761)) >> np.uint64(13)) & np.uint64(0xFF)).astype(np.uint8).tobytes()


def payload(spec) -> bytes:
    kind = spec[0]
    if kind == "fill":
        return bytes([spec[1]]) * spec[2]
    if kind == "pat":
        return pattern(spec[2], spec[1])
    raise ValueError(spec)


def build(sc) -> tuple[bytes, int]:
    w = W.WalWriter(sc["map_bits"])
    for tag, spec in sc["entries"]:
        w.write(tag, payload(spec))
    img = bytearray(w.image())
    end = w.pos
    for op in sc.get("corrupt", []):
        kind = op[0]
        if kind == "xor":         # ("xor", byte position, mask)
            img[op[1]] ^= op[2]
        elif kind == "put32":     # ("put32", position, value): little-endian u32
            img[op[1]:op[1] + 4] = struct.pack("<I", op[2])
        elif kind == "put64":
            img[op[1]:op[1] + 8] = struct.pack("<Q", op[2])
        elif kind == "truncate":  # ("truncate", new size): the file ends early, writer pos kept
            del img[op[1]:]
        elif kind == "zero":      # ("zero", start, stop)
            img[op[1]:op[2]] = bytes(op[2] - op[1])
        else:
            raise ValueError(op)
    if "end_pos" in sc:
        end = sc["end_pos"]
    return bytes(img), end


def iterate(img: bytes, end_pos: int, map_bits: int):
    """WalIterator over WalReader::try_read (wal.rs:226-346), statuses as oracle/wal.c."""
    msize = 1 << map_bits

    def byte_at(i):
        return img[i] if i < len(img) else 0

    def try_read(p):
        base = p & ~(msize - 1)
        boff = p - base
        if msize - boff < 16:                       # read_header: buffer too small
            return None
        hdr = bytes(byte_at(p + k) for k in range(16))
        comb = int.from_bytes(hdr, "little")        # split_header
        crc, ln, tag = comb & ((1 << 64) - 1), (comb >> 64) & 0xFFFFFFFF, comb >> 96
        if ln == 0:
            if crc == 0:
                return None
            return (tag, 0, O.WAL_NONZERO_CRC_LEN0)     # panic "Non-zero crc at len 0"
        if ln < 16 or boff + ln > msize:
            return (tag, 0, O.WAL_BAD_LENGTH)            # Bytes::slice panics
        data = bytes(byte_at(i) for i in range(p + 16, p + ln))
        st = O.WAL_OK if zlib.crc32(data) == crc else O.WAL_CRC_MISMATCH
        return (tag, ln - 16, st)

    out = []
    position = 0
    while position is not None:
        def try_position(p):
            if p >= end_pos:
                return None
            return try_read(p)
        r = try_position(position)
        at = position
        if r is None and position != (position & ~(msize - 1)):   # not first_in_map
            at = (position & ~(msize - 1)) + msize                  # next_start_offset
            r = try_position(at)
        if r is None:
            break
        tag, plen, st = r
        out.append((at, tag, plen, st))
        position = None if st != O.WAL_OK else at + plen + 16
    return out


def scenarios():
    T = W.MAP_BITS_TEST
    M = 1 << T
    sc = []
    # wal.rs:380-446 test_wal (one .. four, tags 5/10/15/20; `two` fills a whole map)
    sc.append({"name": "ref_test_wal", "map_bits": T,
               "entries": [[5, ["fill", 1, 1024]], [10, ["fill", 2, M - 16]], [15, ["fill", 3, 15]],
                           [20, ["fill", 4, 18]]]})
    # wal.rs:448-473: the iterator reaches 4 bytes before the end of a map (no room for a header)
    sc.append({"name": "ref_iterator_over_map_boundary", "map_bits": T,
               "entries": [[1, ["fill", 5, M - 16 - 4]], [2, ["fill", 5, M - 16 - 4]]]})
    # ragged mix over many maps, empty payloads included
    rng = np.random.default_rng(215)
    mix = [[int(rng.integers(1, 6)), ["pat", int(i), int(rng.integers(0, 3000))]] for i in range(600)]
    mix += [[1, ["pat", 9001, 0]], [2, ["pat", 9002, M - 16]], [3, ["pat", 9003, 1]]]
    sc.append({"name": "ragged_mix", "map_bits": T, "entries": mix})
    # production map size, block-sized entries
    sc.append({"name": "production_maps", "map_bits": W.MAP_BITS_PRODUCTION,
               "entries": [[1, ["pat", 100 + i, 9461]] for i in range(40)] + [[2, ["pat", 77, 70000]]]})
    small = [[1 + (i % 5), ["pat", 500 + i, 100 + 37 * i]] for i in range(40)]
    # failures: the iteration stops at (and reports) the first failing entry
    base, _ = build({"map_bits": T, "entries": small})
    pos, _end = O.wal_layout([100 + 37 * i for i in range(40)], T)
    p = [int(x) for x in pos]
    sc.append({"name": "crc_mismatch_payload", "map_bits": T, "entries": small, "corrupt": [["xor", p[17] + 40, 0x10]]})
    sc.append({"name": "crc_mismatch_header", "map_bits": T, "entries": small, "corrupt": [["xor", p[3] + 1, 0x01]]})
    sc.append({"name": "crc_high_bits", "map_bits": T, "entries": small, "corrupt": [["xor", p[5] + 4, 0x80]]})
    sc.append({"name": "len_below_header", "map_bits": T, "entries": small, "corrupt": [["put32", p[9] + 8, 7]]})
    sc.append({"name": "len_past_map", "map_bits": T, "entries": small, "corrupt": [["put32", p[9] + 8, M]]})
    sc.append({"name": "len0_nonzero_crc", "map_bits": T, "entries": small,
               "corrupt": [["put32", p[12] + 8, 0]]})
    sc.append({"name": "len0_zero_crc_mid_map", "map_bits": T, "entries": small,
               "corrupt": [["put32", p[12] + 8, 0], ["put64", p[12], 0]]})
    sc.append({"name": "end_pos_mid", "map_bits": T, "entries": small, "end_pos": p[21]})
    sc.append({"name": "end_pos_inside_entry", "map_bits": T, "entries": small, "end_pos": p[21] + 5})
    sc.append({"name": "truncated_file", "map_bits": T, "entries": small, "corrupt": [["truncate", p[30] + 50]]})
    # a zeroed map start ends the iteration (first_in_map, wal.rs:321-326); entries after it are not read
    big = [[1, ["pat", 700 + i, 5000]] for i in range(40)]
    pb, _ = O.wal_layout([5000] * 40, T)
    first_in_map2 = next(int(x) for x in pb if int(x) == 2 * M)
    sc.append({"name": "zero_map_start", "map_bits": T, "entries": big,
               "corrupt": [["zero", first_in_map2, first_in_map2 + 16]]})
    sc.append({"name": "empty", "map_bits": T, "entries": []})
    return sc


def main() -> None:
    crc = []
    for n in list(range(0, 260)) + [1000, 4096, 4097, 65536, 1 << 20]:
        crc.append({"pat_seed": n % 7, "len": n, "crc": zlib.crc32(pattern(n, n % 7))})
    crc.append({"ascii": "123456789", "crc": zlib.crc32(b"123456789")})  # the CRC-32 check value
    out = {"note": "crc32fast::hash vectors (zlib.crc32) and WalReader iteration scenarios; "
                   "generated by oracle/gen_wal_fixtures.py",
           "crc32": crc, "scenarios": []}
    for sc in scenarios():
        img, end = build(sc)
        exp = iterate(img, end, sc["map_bits"])
        cpos, ctag, clen, cst = O.wal_iter(np.frombuffer(img, dtype=np.uint8), end, sc["map_bits"])
        got = list(zip(cpos.tolist(), ctag.tolist(), clen.tolist(), cst.tolist()))
        assert got == [tuple(x) for x in exp], (sc["name"], got[:5], exp[:5])
        sc = dict(sc)
        sc["image_bytes"] = len(img)
        sc["image_sha256"] = hashlib.sha256(img).hexdigest()
        sc["iter_end"] = end
        sc["expect"] = [list(x) for x in exp]
        out["scenarios"].append(sc)
        print(f"{sc['name']:32s} {len(img):9d} B  {len(exp):4d} entries  last status "
              f"{exp[-1][3] if exp else '-'}")
    with open(OUT, "w") as f:
        json.dump(out, f, separators=(",", ":"))
    print("wrote", OUT, os.path.getsize(OUT), "bytes")


if __name__ == "__main__":
    main()
