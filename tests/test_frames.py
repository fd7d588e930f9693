"""CPU: mv_frame_blocks, the host-side walk of received NetworkMessage frames
(Network::handle_read_stream, network.rs:400-447): a u32 big-endian size, then
bincode(NetworkMessage) (network.rs:36-46), a size of 0 being a ping with 8 more bytes. The
blocks of Blocks / RequestBlocksResponse messages come out as (offset, length) pairs into the
buffer; every other message is skipped; the stream conditions on which the reference drops the
connection return -1. The frames are built here from the bincode rules (enum tag u32 LE, Vec as
u64 LE count, Data<T> as u64 LE length + bytes, data.rs:67-96)."""
import struct

import numpy as np
import pytest

import mysticeti_amd as M

TAG_SUBSCRIBE, TAG_BLOCKS, TAG_REQUEST, TAG_RESPONSE, TAG_NOT_FOUND = range(5)


def frame(body: bytes) -> bytes:
    return struct.pack(">I", len(body)) + body


def blocks_msg(tag: int, blocks) -> bytes:
    out = struct.pack("<IQ", tag, len(blocks))
    for b in blocks:
        out += struct.pack("<Q", len(b)) + b
    return out


def ref(a: int, r: int) -> bytes:  # BlockReference: authority, round, digest (u64 32 + 32 B)
    return struct.pack("<QQQ", a, r, 32) + bytes([a]) * 32


def ping() -> bytes:
    return struct.pack(">I", 0) + struct.pack("<q", 12345)


def listed(buf: bytes):
    offs, lens, consumed = M.frame_blocks(buf)
    return [buf[int(o):int(o) + int(n)] for o, n in zip(offs, lens)], consumed


def test_blocks_come_out_in_stream_order_and_other_messages_are_skipped():
    rng = np.random.default_rng(3)
    blks = [rng.integers(0, 256, size=int(rng.integers(0, 700)), dtype=np.uint8).tobytes() for _ in range(9)]
    stream = (frame(struct.pack("<IQ", TAG_SUBSCRIBE, 17))
              + frame(blocks_msg(TAG_BLOCKS, blks[:3]))
              + ping()
              + frame(struct.pack("<IQ", TAG_REQUEST, 2) + ref(1, 5) + ref(2, 5))
              + frame(blocks_msg(TAG_RESPONSE, blks[3:5]))
              + frame(blocks_msg(TAG_BLOCKS, []))
              + frame(struct.pack("<IQ", TAG_NOT_FOUND, 1) + ref(3, 9))
              + frame(blocks_msg(TAG_BLOCKS, blks[5:]) + b"trailing bytes are allowed"))
    got, consumed = listed(stream)
    assert got == blks and consumed == len(stream)


def test_an_incomplete_trailing_frame_waits_for_more_bytes():
    a, b = b"\x01" * 40, b"\x02" * 50
    whole = frame(blocks_msg(TAG_BLOCKS, [a])) + frame(blocks_msg(TAG_BLOCKS, [b]))
    first = len(frame(blocks_msg(TAG_BLOCKS, [a])))
    for cut in range(first, len(whole)):
        got, consumed = listed(whole[:cut])
        assert got == [a] and consumed == first, cut
    assert listed(whole[:3]) == ([], 0)  # not even a size word
    assert listed(ping()[:7]) == ([], 0)  # a ping's 8 bytes not all there
    assert listed(b"") == ([], 0)


def test_cap_smaller_than_the_count_writes_the_first_and_counts_all():
    blks = [bytes([k]) * (k + 1) for k in range(6)]
    buf = np.frombuffer(frame(blocks_msg(TAG_BLOCKS, blks)), dtype=np.uint8)
    lib = M.load_library()
    off = np.zeros(2, dtype=np.uint64)
    ln = np.zeros(2, dtype=np.uint64)
    n = lib.mv_frame_blocks(M._p(buf), buf.size, M._p(off), M._p(ln), 2, None)
    assert n == 6 and [int(x) for x in ln] == [1, 2]


@pytest.mark.parametrize("case", ["oversize", "tag", "count", "length", "no_tag"])
def test_streams_the_reference_drops(case):
    good = frame(blocks_msg(TAG_BLOCKS, [b"\x05" * 30]))
    if case == "oversize":  # size above MAX_SIZE (network.rs:216-221)
        bad = struct.pack(">I", (16 << 20) + 1) + b"\0" * 8
    elif case == "tag":  # no such NetworkMessage variant
        bad = frame(struct.pack("<IQ", 5, 0))
    elif case == "count":  # more blocks than the frame holds
        bad = frame(struct.pack("<IQ", TAG_BLOCKS, 2) + struct.pack("<Q", 4) + b"abcd")
    elif case == "length":  # a block longer than the rest of its frame
        bad = frame(struct.pack("<IQ", TAG_BLOCKS, 1) + struct.pack("<Q", 99) + b"short")
    else:  # a frame too short for the message tag
        bad = frame(b"\x01\x00")
    with pytest.raises(M.MvError):
        M.frame_blocks(good + bad)
    # the same frames before the bad one are fine on their own
    assert len(listed(good)[0]) == 1
