"""WAL replay check: crc32fast::hash and WalReader iteration
(mysticeti-core/src/wal.rs:146-346).

CPU tests pin the oracle (oracle/wal.c) to tests/golden/wal.json: crc32 vectors from zlib and
iteration scenarios that include the reference's own wal.rs tests (test_wal,
test_wal_iterator_over_map_boundary). GPU tests hold mv_crc32 / mv_wal_verify /
mv_dev_wal_verify bit-exact to the golden expectations and to the oracle.
"""
import hashlib
import struct
import zlib

import numpy as np
import pytest

import gen_wal_fixtures as G
import oracle as O
import wal as W


@pytest.fixture(scope="module")
def fx(golden):
    return golden("wal.json")


# ------------------------------------------------------------------------------------- CPU
def test_oracle_crc32_vectors(fx):
    for v in fx["crc32"]:
        data = v["ascii"].encode() if "ascii" in v else G.pattern(v["len"], v["pat_seed"])
        assert O.crc32(data) == v["crc"], v            # PCLMULQDQ folding (crc32fast's x86_64 path)
        assert O.crc32_table(data) == v["crc"], v      # byte-at-a-time table
        assert zlib.crc32(data) == v["crc"]


def test_scenario_images_and_oracle_iteration(fx):
    names = [sc["name"] for sc in fx["scenarios"]]
    assert "ref_test_wal" in names and "ref_iterator_over_map_boundary" in names
    for sc in fx["scenarios"]:
        img, end = G.build(sc)
        assert hashlib.sha256(img).hexdigest() == sc["image_sha256"], sc["name"]
        assert end == sc["iter_end"]
        pos, tag, ln, st = O.wal_iter(np.frombuffer(img, dtype=np.uint8), end, sc["map_bits"])
        got = [list(x) for x in zip(pos.tolist(), tag.tolist(), ln.tolist(), st.tolist())]
        assert got == sc["expect"], sc["name"]


def test_reference_test_wal_positions(fx):
    """wal.rs:380-446: `two` (MAP_SIZE - 16 bytes) cannot share a map with `one`, so it starts at
    the next map; the iterator returns one, two, three, four with their tags, then None."""
    sc = next(s for s in fx["scenarios"] if s["name"] == "ref_test_wal")
    M = 1 << sc["map_bits"]
    assert [e[0] for e in sc["expect"]] == [0, M, 2 * M, 2 * M + 15 + 16]
    assert [e[1] for e in sc["expect"]] == [5, 10, 15, 20]
    assert [e[2] for e in sc["expect"]] == [1024, M - 16, 15, 18]
    b = next(s for s in fx["scenarios"] if s["name"] == "ref_iterator_over_map_boundary")
    assert b["expect"][1][0] >= M  # assert!(pos2.start >= MAP_SIZE)


def test_layout_matches_writer():
    import mysticeti_amd as M

    rng = np.random.default_rng(3)
    for bits in (8, 12, 16, 24):
        lens = rng.integers(0, (1 << bits) - 16, size=300)
        w = W.WalWriter(bits)
        want = [w.write(1, bytes(int(n))) for n in lens]
        opos, oend = O.wal_layout(lens, bits)
        lpos, lend = M.wal_layout(lens, bits)
        assert opos.tolist() == want and lpos.tolist() == want
        assert oend == lend == w.pos


def test_bench_device_image_matches_host_image():
    """bench_wal builds its WAL image in HBM from the distinct entries by contiguous runs; on
    torch's CPU device it must give the host builder's bytes (map padding, cycle wraps)."""
    import os
    import sys

    import torch

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench_wal

    rng = np.random.default_rng(11)
    for bits, k, n in ((12, 7, 200), (16, 13, 500), (14, 1, 90)):
        payloads = [rng.integers(0, 256, size=int(rng.integers(1, 900)), dtype=np.uint8).tobytes() for _ in range(k)]
        img, pos, lens, end = bench_wal.build_image(payloads, n, bits)
        d_img, dpos, dlens, dend = bench_wal.build_image_device(payloads, n, bits, torch, torch.device("cpu"))
        assert dend == end and dpos.tolist() == pos.tolist() and dlens.tolist() == lens.tolist()
        assert bytes(d_img.numpy()) == bytes(img)


def test_header_combine_split():
    """wal.rs:511-521: header = crc | len << 64 | tag << 96, little-endian."""
    for crc in (0, 1, 12, (1 << 64) - 1):
        for ln in (0, 1, 18, (1 << 32) - 1):
            for tag in (0, 1, 18, (1 << 32) - 1):
                h = W.header(crc, ln, tag)
                v = int.from_bytes(h, "little")
                assert (v & ((1 << 64) - 1), (v >> 64) & 0xFFFFFFFF, v >> 96) == (crc, ln, tag)


# ------------------------------------------------------------------------------------- GPU
@pytest.mark.gpu
def test_gpu_crc32_vectors(engine, fx):
    items = [v["ascii"].encode() if "ascii" in v else G.pattern(v["len"], v["pat_seed"]) for v in fx["crc32"]]
    got = engine.crc32(items)
    assert got.tolist() == [v["crc"] for v in fx["crc32"]]


@pytest.mark.gpu
def test_gpu_crc32_ragged_offsets(engine):
    """Every start and end alignment, lengths across the row (256 B) and prefix boundaries."""
    rng = np.random.default_rng(7)
    buf = rng.integers(0, 256, size=1 << 20, dtype=np.uint8)
    offs, lens = [], []
    for a in range(0, 8):
        for n in list(range(0, 70)) + [250, 251, 252, 253, 254, 255, 256, 257, 260, 508, 509, 511, 512, 513,
                                       1023, 1024, 1025, 4099, 65537]:
            offs.append(a + 8 * len(offs))
            lens.append(n)
    offs = np.array(offs, dtype=np.uint64) % np.uint64(len(buf) - 70000)
    lens = np.array(lens, dtype=np.uint64)
    got = engine.crc32_packed(buf, offs, lens)
    want = O.crc32_batch(buf, offs, lens)
    assert (got == want).all()
    assert int(got[5]) == zlib.crc32(buf[int(offs[5]):int(offs[5]) + int(lens[5])].tobytes())


@pytest.mark.gpu
def test_gpu_wal_scenarios(engine, fx):
    for sc in fx["scenarios"]:
        img, end = G.build(sc)
        pos, tag, ln, st = engine.wal_verify(img, end, sc["map_bits"])
        got = [list(x) for x in zip(pos.tolist(), tag.tolist(), ln.tolist(), st.tolist())]
        assert got == sc["expect"], sc["name"]


@pytest.mark.gpu
def test_gpu_wal_iter_until_reference_semantics(engine, fx):
    sc = next(s for s in fx["scenarios"] if s["name"] == "ref_test_wal")
    img, end = G.build(sc)
    items = list(engine.wal_iter_until(img, end, sc["map_bits"]))
    M = 1 << sc["map_bits"]
    assert [(p, t) for p, (t, _) in items] == [(0, 5), (M, 10), (2 * M, 15), (2 * M + 31, 20)]
    assert items[1][1][1] == bytes([2]) * (M - 16) and items[3][1][1] == bytes([4]) * 18
    bad = next(s for s in fx["scenarios"] if s["name"] == "crc_mismatch_payload")
    img, end = G.build(bad)
    it = engine.wal_iter_until(img, end, bad["map_bits"])
    with pytest.raises(Exception, match="Crc mismatch, expected"):
        for _ in it:
            pass
    z = next(s for s in fx["scenarios"] if s["name"] == "len0_nonzero_crc")
    img, end = G.build(z)
    with pytest.raises(Exception, match="Non-zero crc at len 0"):
        list(engine.wal_iter_until(img, end, z["map_bits"]))


@pytest.mark.gpu
def test_gpu_wal_fuzz_against_oracle(engine):
    """Random WALs (test and small maps) with random single corruptions, against the oracle."""
    rng = np.random.default_rng(11)
    for trial in range(40):
        bits = int(rng.choice([10, 12, 16]))
        w = W.WalWriter(bits)
        for i in range(int(rng.integers(1, 300))):
            n = int(rng.integers(0, min(3000, (1 << bits) - 16) + 1))
            w.write(int(rng.integers(0, 6)), rng.integers(0, 256, size=n, dtype=np.uint8).tobytes())
        img = bytearray(w.image())
        end = w.pos
        kind = trial % 5
        if kind == 1 and img:      # flip a random byte anywhere
            img[int(rng.integers(0, len(img)))] ^= 1 << int(rng.integers(0, 8))
        elif kind == 2 and img:    # truncate the file
            img = img[:int(rng.integers(0, len(img)))]
        elif kind == 3:            # iterate up to an earlier writer position
            end = int(rng.integers(0, end + 1))
        elif kind == 4 and len(img) > 16:  # overwrite a random u32 with a random length
            p = int(rng.integers(0, len(img) - 4))
            img[p:p + 4] = struct.pack("<I", int(rng.integers(0, 1 << 17)))
        img = bytes(img)
        want = O.wal_iter(np.frombuffer(img, dtype=np.uint8), end, bits)
        got = engine.wal_verify(img, end, bits)
        for g, e in zip(got, want):
            assert g.tolist() == e.tolist(), (trial, kind)


@pytest.mark.gpu
def test_gpu_wal_block_entries_production_maps(engine):
    """Config-4-sized entries (9,461-byte block bincode) and a near-map-size entry at 16 MiB maps."""
    rng = np.random.default_rng(5)
    w = W.WalWriter(W.MAP_BITS_PRODUCTION)
    payloads = [rng.integers(0, 256, size=9461, dtype=np.uint8).tobytes() for _ in range(64)]
    for i in range(4000):
        w.write(1, payloads[i % 64])
    w.write(4, rng.integers(0, 256, size=(1 << 24) - 16, dtype=np.uint8).tobytes())  # a whole map
    for i in range(100):
        w.write(2, payloads[i % 64][:100 + i])
    img = w.image()
    pos, tag, ln, st = engine.wal_verify(img, w.pos, W.MAP_BITS_PRODUCTION)
    opos, otag, oln, ost = O.wal_iter(np.frombuffer(img, dtype=np.uint8), w.pos, W.MAP_BITS_PRODUCTION)
    assert len(pos) == 4101 and (st == 0).all()
    assert pos.tolist() == opos.tolist() and ln.tolist() == oln.tolist() and tag.tolist() == otag.tolist()


@pytest.mark.gpu
def test_gpu_wal_dense_maps_second_walk(engine):
    """Maps holding more entries than the walk's first per-map guess (4,096): the second walk
    writes each map's records at its own offset (no maps x max-count buffer), as the reference
    iterates them (wal.rs:226-346)."""
    rng = np.random.default_rng(12)
    w = W.WalWriter(W.MAP_BITS_PRODUCTION)
    for i in range(9000):  # ~60 B entries: two maps hold > 4,096 each
        w.write(i % 5, rng.integers(0, 256, size=int(rng.integers(0, 64)), dtype=np.uint8).tobytes())
    w.write(3, rng.integers(0, 256, size=(1 << 24) - 100, dtype=np.uint8).tobytes())  # forces a map change
    for i in range(5000):
        w.write(1, rng.integers(0, 256, size=40, dtype=np.uint8).tobytes())
    img = w.image()
    pos, tag, ln, st = engine.wal_verify(img, w.pos, W.MAP_BITS_PRODUCTION)
    opos, otag, oln, ost = O.wal_iter(np.frombuffer(img, dtype=np.uint8), w.pos, W.MAP_BITS_PRODUCTION)
    assert len(pos) == 14001 and (st == 0).all()
    assert pos.tolist() == opos.tolist() and ln.tolist() == oln.tolist() and tag.tolist() == otag.tolist()


@pytest.mark.gpu
def test_gpu_dev_wal_and_crc(engine):
    import torch

    w = W.WalWriter(16)
    rng = np.random.default_rng(9)
    for i in range(500):
        w.write(1 + i % 3, rng.integers(0, 256, size=int(rng.integers(0, 5000)), dtype=np.uint8).tobytes())
    img = np.frombuffer(w.image(), dtype=np.uint8)
    d_img = torch.from_numpy(img.copy()).cuda()
    cap = 600
    d_pos = torch.zeros(cap, dtype=torch.int64, device="cuda")
    d_tag = torch.zeros(cap, dtype=torch.int32, device="cuda")
    d_len = torch.zeros(cap, dtype=torch.int32, device="cuda")
    d_st = torch.zeros(cap, dtype=torch.uint8, device="cuda")
    n = engine.dev_wal_verify(0, d_img, img.size, w.pos, 16, d_pos, d_tag, d_len, d_st, cap)
    opos, otag, oln, ost = O.wal_iter(img, w.pos, 16)
    assert n == len(opos) == 500
    assert d_pos.cpu().numpy()[:n].astype(np.uint64).tolist() == opos.tolist()
    assert (d_st.cpu().numpy()[:n] == 0).all()
    # mv_dev_crc32 over the payloads in place
    d_off = torch.from_numpy((opos + 16).astype(np.int64)).cuda()
    d_ln = torch.from_numpy(oln.astype(np.int64)).cuda()
    d_out = torch.zeros(n, dtype=torch.int32, device="cuda")
    engine.dev_crc32(0, d_img, d_off, d_ln, n, d_out)
    torch.cuda.synchronize()
    want = O.crc32_batch(img, opos + 16, oln.astype(np.uint64))
    assert (d_out.cpu().numpy().view(np.uint32) == want).all()
