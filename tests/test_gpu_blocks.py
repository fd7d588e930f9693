"""GPU: StatementBlock::verify through mv_verify_blocks — statuses in the reference's error
order (types.rs:315-376) and both Blake2b digests bit-exact vs the fixtures and the oracle."""
import hashlib

import numpy as np
import pytest

import blocks as B
import oracle as O

pytestmark = pytest.mark.gpu


def committee_arrays(c):
    pks = np.frombuffer(b"".join(bytes.fromhex(x) for x in c["pks"]), dtype=np.uint8).reshape(-1, 32)
    return pks, np.array(c["stakes"], dtype=np.uint64), c["epoch"]


def test_block_edge_cases(engine, golden):
    e = golden("block_edge.json")
    pks, stakes, epoch = committee_arrays(e["committee"])
    ok = engine.set_committee(pks, stakes, epoch)
    assert ok.all()
    blocks = [bytes.fromhex(c["bincode"]) for c in e["cases"]]
    st, md, bd = engine.verify_blocks(blocks)
    for c, s, b, m, d in zip(e["cases"], st, blocks, md, bd):
        assert int(s) == c["status"], c["note"]
        if c["status"] != 1:
            ost, omd, obd = O.block_verify(b, pks, stakes, epoch)
            assert m.tobytes() == omd and d.tobytes() == obd, c["note"]


def test_config1_4096_blocks(engine, golden):
    g = golden("blocks_config1.json")
    pks, stakes, epoch = committee_arrays(g["committee"])
    engine.set_committee(pks, stakes, epoch)
    blks = B.gen_config1(O.sign)
    bins = [b.bincode() for b in blks]
    assert hashlib.sha256(b"".join(bins)).hexdigest() == g["sha256_bincode_concat"]
    st, md, bd = engine.verify_blocks(bins)
    assert (st == 0).all()
    assert hashlib.sha256(md.tobytes()).hexdigest() == g["sha256_msg_digests"]
    assert hashlib.sha256(bd.tobytes()).hexdigest() == g["sha256_block_digests"]


def test_config4_shape_blocks(engine, golden):
    g = golden("blocks_config4_sample.json")
    pks, stakes, epoch = committee_arrays(g["committee"])
    engine.set_committee(pks, stakes, epoch)
    blks = B.gen_config4(O.sign, rounds=2)
    bins = [b.bincode() for b in blks]
    st, md, bd = engine.verify_blocks(bins)
    assert (st == 0).all()
    assert hashlib.sha256(md.tobytes()).hexdigest() == g["sha256_msg_digests"]
    assert hashlib.sha256(bd.tobytes()).hexdigest() == g["sha256_block_digests"]


def test_mixed_lengths_and_failures(engine):
    """Ragged pre-image lengths in one wave (41 B .. ~9 KB) with failures mixed in."""
    seeds = [B.authority_seed(a) for a in range(7)]
    pks = np.frombuffer(b"".join(O.public_key(s) for s in seeds), dtype=np.uint8).reshape(-1, 32)
    stakes = np.array([3, 1, 1, 2, 1, 1, 1], dtype=np.uint64)
    engine.set_committee(pks, stakes, 0)
    prev = [B.genesis(a) for a in range(7)]
    blocks = []
    rng = np.random.default_rng(5)
    for r in range(1, 40):
        for a in range(7):
            k = int(rng.integers(1, 8))
            inc = [prev[a].reference()] + [prev[x].reference() for x in range(7) if x != a][: k - 1]
            sts = [("share", bytes(int(rng.integers(0, 700))))] * int(rng.integers(0, 3))
            sts += [("range", prev[(a + 1) % 7].reference(), 0, int(rng.integers(0, 5)))] * int(rng.integers(0, 20))
            blocks.append(B.new_with_signer(a, r, inc, sts, r, False, 0, seeds[a], O.sign))
        prev = blocks[-7:]
    bins = [b.bincode() for b in blocks]
    # corrupt a few
    bins[3] = bins[3][:-5] + bytes([bins[3][-5] ^ 1]) + bins[3][-4:]
    bins[10] = bins[10][:60]
    st, md, bd = engine.verify_blocks(bins)
    for i, b in enumerate(bins):
        ost, omd, obd = O.block_verify(b, pks, stakes, 0)
        assert int(st[i]) == ost, i
        if ost != 1:
            assert md[i].tobytes() == omd and bd[i].tobytes() == obd, i
    assert len({int(s) for s in st}) >= 3


def test_edge_blocks_through_batch_path(engine, golden):
    """>= MV_BATCH_MIN blocks take the batch path: the edge cases tiled 200x keep their
    statuses. Blocks rejected ahead of the signature check (parse error, epoch, unknown
    author, genesis) are taken out of the combined equation, so without the one bad
    signature the batch passes with no fallback; with it, the fallback is exact."""
    import mysticeti_amd as M

    e = golden("block_edge.json")
    pks, stakes, epoch = committee_arrays(e["committee"])
    engine.set_committee(pks, stakes, epoch)
    # the fixture's "bad signature" flips a bit of R, which then does not decode: decided per
    # signature before the combination (no fallback). A flipped bit of s (still < l) with R
    # intact can only be caught by the combined equation, so it forces the fallback.
    valid = bytes.fromhex(next(c for c in e["cases"] if c["note"] == "valid")["bincode"])
    sig = bytearray(valid[-64:])
    sig[40] ^= 0x10
    dig = hashlib.blake2b(M.block_preimage(valid) + bytes(sig), digest_size=32).digest()
    bad_s = {"bincode": (valid[:24] + dig + valid[56:-64] + bytes(sig)).hex(), "status": 6, "note": "s bit flip"}
    for drop_bad_sig in (True, False):
        cases = [c for c in e["cases"] if not c["note"].startswith("bad signature")]
        if not drop_bad_sig:
            cases.append(bad_s)
        reps = M.BATCH_MIN // len(cases) + 1
        blocks = [bytes.fromhex(c["bincode"]) for c in cases] * reps
        b0, f0 = engine.batch_stats()
        st, md, bd = engine.verify_blocks(blocks)
        b1, f1 = engine.batch_stats()
        assert [int(x) for x in st] == [c["status"] for c in cases] * reps
        assert b1 - b0 == 1
        assert f1 - f0 == (0 if drop_bad_sig else 1)


def test_tampered_blocks_stay_out_of_the_batch_equation(engine, golden):
    """A block whose digest does not match is DIGEST_MISMATCH whatever its signature
    (types.rs:327-332 before :346-348). Tampered blocks -- s flipped with the digest left
    stale, or a pre-image byte changed -- are taken out of the combined equation after the
    hashes, so 4,096 blocks with tampered ones pass the batch with no fallback."""
    g = golden("blocks_config1.json")
    pks, stakes, epoch = committee_arrays(g["committee"])
    engine.set_committee(pks, stakes, epoch)
    bins = [b.bincode() for b in B.gen_config1(O.sign)]
    t1 = bytearray(bins[17])
    t1[-20] ^= 0x04  # s bit: invalid signature, stale digest
    t2 = bytearray(bins[2222])
    t2[-64 - 8 - 8 - 1 - 3] ^= 0x01  # meta_creation_time_ns byte: new message, stale digest
    bins[17], bins[2222] = bytes(t1), bytes(t2)
    b0, f0 = engine.batch_stats()
    st, md, bd = engine.verify_blocks(bins)
    b1, f1 = engine.batch_stats()
    assert b1 - b0 == 1 and f1 - f0 == 0
    assert st[17] == 2 and st[2222] == 2 and (np.delete(st, [17, 2222]) == 0).all()
    for i in (17, 2222):
        ost, omd, obd = O.block_verify(bins[i], pks, stakes, epoch)
        assert ost == 2 and md[i].tobytes() == omd and bd[i].tobytes() == obd


def test_config4_shape_4100_blocks_through_the_batch_path(engine):
    """4,100 config-4-shaped blocks (100 validators, 67 includes, 512-B tx, 66 VoteRanges)
    take the batch path: every verdict and digest matches the oracle's on a sample and on
    every tampered block; blocks whose signature is bad under a correct digest fail the
    equation of their sub-batch only and are re-verified exactly."""
    import hashlib as H

    import mysticeti_amd as M
    import mysticeti_amd.blocks as MB

    base = MB.config4(engine, rounds=41)
    pks, stakes = MB.committee(engine, 100, distinct=True)
    engine.set_committee(pks, stakes, 0)
    bins = list(base)
    # bad signature, digest recomputed over the bad signature: SIG_INVALID, caught by the equation
    for i in (7, 2900):
        b = bytearray(bins[i])
        b[-20] ^= 0x10
        pre = M.block_preimage(bytes(b))
        b[24:56] = H.blake2b(pre + bytes(b[-64:]), digest_size=32).digest()
        bins[i] = bytes(b)
    t = bytearray(bins[1000])
    t[-20] ^= 0x10  # stale digest: DIGEST_MISMATCH, kept out of the equation
    bins[1000] = bytes(t)
    c0 = engine.batch_counters()
    st, md, bd = engine.verify_blocks(bins)
    d = [b - a for a, b in zip(c0, engine.batch_counters())]
    assert d[0] == 1 and d[1] == 1 and d[3] >= 1  # one batch; the failing groups hold blocks 7, 2900
    want = np.zeros(len(bins), np.uint8)
    want[[7, 2900]] = 6
    want[1000] = 2
    assert (st == want).all()
    rng = np.random.default_rng(4)
    sample = sorted(set(rng.choice(len(bins), 40, replace=False).tolist()) | {7, 1000, 2900})
    for i in sample:
        ost, omd, obd = O.block_verify(bins[i], pks, stakes, 0)
        assert int(st[i]) == ost and md[i].tobytes() == omd and bd[i].tobytes() == obd, i


@pytest.mark.parametrize("split", ["1", "0"])
def test_comb_split_and_fused_paths_agree(engine, golden, opts, split):
    """Batches under MV_BATCH_MIN take the committee comb verify. Long blocks run it split
    (k_comb_pre -- s < l, R decode, R - [s]B -- on a second stream beside the hash, k_comb_post
    after it); MV_COMB_SPLIT_BYTES=1 forces the split for every block, 0 the fused kernel: the
    edge cases, ragged lengths and config-4-shaped blocks with bad signatures keep the oracle's
    verdicts and digests either way. (The queue's kernels: the resident service is off here.)"""
    import hashlib as H

    import mysticeti_amd as M
    import mysticeti_amd.blocks as MB

    opts("MV_COMB_SPLIT_BYTES", int(split))
    opts("MV_ONLINE", 0)
    test_block_edge_cases(engine, golden)
    test_mixed_lengths_and_failures(engine)
    bins = list(MB.config4(engine, rounds=1))[:64]
    pks, stakes = MB.committee(engine, 100, distinct=True)
    engine.set_committee(pks, stakes, 0)
    for i, flip in ((5, -20), (33, -50)):  # s bit (s < l), R bit; digest recomputed: SIG_INVALID
        b = bytearray(bins[i])
        b[flip] ^= 0x10
        b[24:56] = H.blake2b(M.block_preimage(bytes(b)) + bytes(b[-64:]), digest_size=32).digest()
        bins[i] = bytes(b)
    st, md, bd = engine.verify_blocks(bins)
    assert st[5] == 6 and st[33] == 6 and (np.delete(st, [5, 33]) == 0).all()
    for i in (0, 5, 33, 63):
        ost, omd, obd = O.block_verify(bins[i], pks, stakes, 0)
        assert int(st[i]) == ost and md[i].tobytes() == omd and bd[i].tobytes() == obd, i


def test_pinned_caller_buffer_is_read_in_place(engine):
    """Blocks in page-locked caller memory (mv_host_alloc), packed in order, are DMAd in
    place (no host pack) once a chunk exceeds the zero-copy size, at any alignment; the verdicts
    and digests equal the pageable path's, including a tampered block."""
    import mysticeti_amd.blocks as MB

    base = MB.config4(engine, rounds=3)  # 300 blocks, ~2.8 MB
    pks, stakes = MB.committee(engine, 100, distinct=True)
    engine.set_committee(pks, stakes, 0)
    bins = list(base)
    t = bytearray(bins[123])
    t[-5] ^= 1
    bins[123] = bytes(t)
    offs, pos = [], 0
    for b in bins:
        offs.append(pos)
        pos += len(b) + (len(offs) % 3)  # packed back to back, with 0-2 byte gaps: any alignment
    flat = np.zeros(pos + 64, np.uint8)
    for o, b in zip(offs, bins):
        flat[o:o + len(b)] = np.frombuffer(b, np.uint8)
    off = np.array(offs, np.uint64)
    ln = np.array([len(b) for b in bins], np.uint64)
    st0, md0, bd0 = engine.verify_blocks_packed(flat, off, ln)
    pinned = engine.host_empty(flat.shape)
    try:
        pinned[:] = flat
        st1, md1, bd1 = engine.verify_blocks_packed(pinned, off, ln)
    finally:
        engine.host_free(pinned)
    assert (st0 == st1).all() and (md0 == md1).all() and (bd0 == bd1).all()
    assert int(st1[123]) != 0 and (np.delete(st1, 123) == 0).all()
    ost, omd, obd = O.block_verify(bins[123], pks, stakes, 0)
    assert int(st1[123]) == ost and md1[123].tobytes() == omd and bd1[123].tobytes() == obd


def test_batch_call_in_two_halves_matches_small_calls(engine):
    """8,300 config-4-shaped blocks in one call (both halves >= MV_BATCH_MIN: the parse of the second
    half runs on another stream beside the hash of the first, engine.cpp enqueue_blocks), with
    tampered and truncated blocks in both halves: every verdict and digest equals the one the
    same block gets in 64-block calls (the comb path, held to the oracle by the tests above)."""
    import mysticeti_amd.blocks as MB

    base = MB.config4(engine, rounds=41)
    pks, stakes = MB.committee(engine, 100, distinct=True)
    engine.set_committee(pks, stakes, 0)
    bins = list(base) + list(base) + list(base)[:100]
    for i in (10, 4200, 8100, 8290):  # stale digest
        t = bytearray(bins[i])
        t[-20] ^= 0x10
        bins[i] = bytes(t)
    for i in (3000, 7000):  # truncated
        bins[i] = bins[i][: len(bins[i]) // 2]
    st, md, bd = engine.verify_blocks(bins)
    assert st.shape == (8300,)
    assert (st[[10, 4200, 8100, 8290]] == 2).all() and st[3000] != 0 and st[7000] != 0
    for lo in list(range(0, 256, 64)) + list(range(4096, 4352, 64)) + list(range(7936, 8300, 64)) + [2944, 6976]:
        s2, m2, b2 = engine.verify_blocks(bins[lo:lo + 64])
        assert (s2 == st[lo:lo + 64]).all(), lo
        ok = s2 == 0
        assert (m2[ok] == md[lo:lo + 64][ok]).all() and (b2[ok] == bd[lo:lo + 64][ok]).all(), lo


def test_two_pinned_callers_at_once(engine):
    """Two callers, each with its own page-locked buffer (> the zero-copy size, so each chunk is
    a candidate for the in-place DMA), submit at the same time: a merged pass must not DMA the
    span between the two allocations; verdicts equal the pageable path's."""
    import threading

    import mysticeti_amd.blocks as MB

    base = MB.config4(engine, rounds=3)
    pks, stakes = MB.committee(engine, 100, distinct=True)
    engine.set_committee(pks, stakes, 0)
    bins = list(base)
    t = bytearray(bins[77])
    t[-5] ^= 1
    bins[77] = bytes(t)
    flat, off, ln = MB.pack(bins)
    want = engine.verify_blocks_packed(flat, off, ln)
    bufs = [engine.host_empty(flat.shape) for _ in range(2)]
    try:
        for b in bufs:
            b[:] = flat
        for _ in range(4):
            res = [None, None]

            def run(k):
                res[k] = engine.verify_blocks_packed(bufs[k], off, ln)

            th = [threading.Thread(target=run, args=(k,)) for k in range(2)]
            for x in th:
                x.start()
            for x in th:
                x.join()
            for r in res:
                assert r is not None
                for a, b in zip(r, want):
                    assert (a == b).all()
    finally:
        for b in bufs:
            engine.host_free(b)
    assert int(want[0][77]) != 0 and (np.delete(want[0], 77) == 0).all()


def test_frames_verified_in_place_equal_the_blocks(engine, golden):
    """Received NetworkMessage frames (network.rs:400-447) verified in place: mv_frame_blocks
    lists the Blocks / RequestBlocksResponse messages' blocks, mv_verify_blocks checks them on the
    frame buffer. Statuses and digests equal verify_blocks on the same blocks, a tampered block
    included, with pings and other messages between the frames, at a small and a batch-size
    count (the online service and the batch path)."""
    import struct

    import mysticeti_amd as M

    g = golden("blocks_config1.json")
    pks, stakes, epoch = committee_arrays(g["committee"])
    engine.set_committee(pks, stakes, epoch)
    bins = [b.bincode() for b in B.gen_config1(O.sign)]
    bins[5] = bins[5][:-3] + bytes([bins[5][-3] ^ 1]) + bins[5][-2:]  # a signature byte

    def frame(tag, blks):
        body = struct.pack("<IQ", tag, len(blks)) + b"".join(struct.pack("<Q", len(b)) + b for b in blks)
        return struct.pack(">I", len(body)) + body

    for blocks in (bins[:40], bins):
        stream = b""
        for k in range(0, len(blocks), 37):
            stream += frame(1 if k % 2 == 0 else 3, blocks[k:k + 37])
            stream += struct.pack(">I", 0) + bytes(8)  # a ping
            stream += struct.pack(">I", 12) + struct.pack("<IQ", 0, k)  # SubscribeOwnFrom
        st, md, bd, consumed = engine.verify_frames(stream)
        assert consumed == len(stream)
        want_st, want_md, want_bd = engine.verify_blocks(blocks)
        assert (st == want_st).all() and (md == want_md).all() and (bd == want_bd).all()
        assert int(st[5]) != 0 and (np.delete(st, 5) == 0).all()
