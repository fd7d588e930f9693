"""ORACLE / TEST INFRASTRUCTURE ONLY: a pure-Python WalWriter that builds WAL images for the
tests and the bench corpus (never shipped).

Restates WalWriter::writev (mysticeti-core/src/wal.rs:150-188) and combine_header
(wal.rs:211-216): each entry is a 16-byte little-endian header crc (u64) | len (u32) | tag (u32),
len = payload + 16, crc = crc32fast::hash(payload), and an entry that would straddle a map of
2^map_bits bytes is moved to the next map, the gap zero-filled. The crc comes from zlib.crc32
(the same CRC-32/ISO-HDLC, an independent implementation of crc32fast's function).
"""
from __future__ import annotations

import struct
import zlib

MAP_BITS_PRODUCTION = 24  # wal.rs:95-98 (16 MiB maps)
MAP_BITS_TEST = 16        # wal.rs:99-103 (cfg(test): 64 KiB maps)


def header(crc: int, length: int, tag: int) -> bytes:
    """combine_header(crc, len, tag).to_le_bytes()"""
    return struct.pack("<QII", crc, length, tag)


class WalWriter:
    def __init__(self, map_bits: int = MAP_BITS_TEST, image: bytes = b""):
        self.map_bits = map_bits
        self.buf = bytearray(image)
        self.pos = len(self.buf)

    def _offset(self, p: int) -> int:
        return p & ~((1 << self.map_bits) - 1)

    def writev(self, tag: int, parts) -> int:
        payload = b"".join(bytes(x) for x in parts)
        length = len(payload) + 16
        assert length <= 1 << self.map_bits
        if self._offset(self.pos) != self._offset(self.pos + length - 1):
            extra = self._offset(self.pos + length - 1) - self.pos
            self.buf += bytes(extra)
            self.pos += extra
        position = self.pos
        self.buf += header(zlib.crc32(payload), length, tag) + payload
        self.pos += length
        return position

    def write(self, tag: int, data: bytes) -> int:
        return self.writev(tag, [data])

    def image(self) -> bytes:
        return bytes(self.buf)
