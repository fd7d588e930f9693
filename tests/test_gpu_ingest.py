"""GPU: device-side block ingest. mv_verify_blocks parses the bincode,
builds the pre-image and runs the StatementBlock::verify checks on the GPU (ingest.hip); its
verdicts and digests must equal the host-codec path (MV_FLAG_HOST_PARSE, block_codec.cpp) and
the oracle on every input, malformed and truncated ones included (types.rs:315-376,
data.rs:43-52). mv_dev_verify_blocks runs the same pipeline on HBM-resident bytes."""
import hashlib

import numpy as np
import pytest

import blocks as B
import mysticeti_amd as M
import oracle as O

pytestmark = pytest.mark.gpu


FORM = {"name": ""}


@pytest.fixture(params=["in_comb", "two_kernel", "separate_hash", "batch_walk", "batch_stage"], autouse=True)
def ingest_form(request, opts):
    """Every test runs on the device ingest forms: on small calls the parse and the digests
    inside k_verify_comb16 (the default), k_block_ingest + the digests inside k_verify_comb16
    (MV_INGEST_IN_COMB=0) and k_block_ingest + a separate k_b2_quad launch (MV_HASH_IN_COMB=0);
    at batch size (agree() repeats the inputs to >= MV_BATCH_MIN blocks) the one-pass walk
    (k_block_walk: parse, checks and both digests from the bincode, the default) and the staged
    form (k_block_ingest + k_b2_lane, MV_BLK_WALK=0)."""
    opts("MV_HASH_IN_COMB", request.param != "separate_hash")
    opts("MV_INGEST_IN_COMB", request.param != "two_kernel")
    opts("MV_BLK_WALK", request.param != "batch_stage")
    FORM["name"] = request.param
    return request.param


@pytest.fixture(scope="module")
def host_engine():
    with M.Engine(devices=(0,), host_parse=True) as e:
        yield e


def committee(c):
    pks = np.frombuffer(b"".join(bytes.fromhex(x) for x in c["pks"]), dtype=np.uint8).reshape(-1, 32)
    return pks, np.array(c["stakes"], dtype=np.uint64), c["epoch"]


def agree(engine, host_engine, bins, pks, stakes, epoch):
    engine.set_committee(pks, stakes, epoch)
    host_engine.set_committee(pks, stakes, epoch)
    if FORM["name"].startswith("batch") and len(bins) < M.BATCH_MIN:
        # the batch-size forms: the same blocks repeated to one batch-path call; every copy
        # must get the verdict and digests of the first
        n = len(bins)
        reps = -(-M.BATCH_MIN // n)
        st, md, bd = engine.verify_blocks(bins * reps)
        for r in range(1, reps):
            assert (st[r * n:(r + 1) * n] == st[:n]).all(), r
            ok = st[:n] != M.BLOCK_PARSE_ERROR
            assert (md[r * n:(r + 1) * n][ok] == md[:n][ok]).all() and (bd[r * n:(r + 1) * n][ok] == bd[:n][ok]).all(), r
        st, md, bd = st[:n], md[:n], bd[:n]
    else:
        st, md, bd = engine.verify_blocks(bins)
    hst, hmd, hbd = host_engine.verify_blocks(bins)
    assert (st == hst).all(), np.nonzero(st != hst)[0][:10]
    for i in range(len(bins)):
        if st[i] != M.BLOCK_PARSE_ERROR:
            assert md[i].tobytes() == hmd[i].tobytes() and bd[i].tobytes() == hbd[i].tobytes(), i
    return st, md, bd


def small_committee():
    seeds = [B.authority_seed(a) for a in range(7)]
    pks = np.frombuffer(b"".join(O.public_key(s) for s in seeds), dtype=np.uint8).reshape(-1, 32)
    return pks, np.array([3, 1, 1, 2, 1, 1, 1], dtype=np.uint64)


def test_edge_cases(engine, host_engine, golden):
    e = golden("block_edge.json")
    pks, stakes, epoch = committee(e["committee"])
    bins = [bytes.fromhex(c["bincode"]) for c in e["cases"]]
    st, _, _ = agree(engine, host_engine, bins, pks, stakes, epoch)
    assert [int(s) for s in st] == [c["status"] for c in e["cases"]]


def test_truncations(engine, host_engine):
    pks, stakes = small_committee()
    blk = B.gen_config4(O.sign, rounds=1, n_auth=7, n_inc=5, n_vr=3)[-1].bincode()
    cut = [blk[:k] for k in range(len(blk))]
    st, _, _ = agree(engine, host_engine, cut, pks, stakes, 0)
    assert (st == M.BLOCK_PARSE_ERROR).all()


def test_byte_flips_and_garbage_vs_oracle(engine, host_engine):
    pks, stakes = small_committee()
    base = [b.bincode() for b in B.gen_config4(O.sign, rounds=2, n_auth=7, n_inc=5, n_vr=3)]
    rng = np.random.default_rng(21)
    out = []
    for _ in range(1500):
        b = bytearray(base[int(rng.integers(0, len(base)))])
        for _ in range(int(rng.integers(1, 4))):
            b[int(rng.integers(0, len(b)))] ^= 1 << int(rng.integers(0, 8))
        out.append(bytes(b))
    for _ in range(300):
        out.append(rng.integers(0, 256, size=int(rng.integers(0, 700)), dtype=np.uint8).tobytes())
    out += base
    st, md, bd = agree(engine, host_engine, out, pks, stakes, 0)
    for i in range(0, len(out), 5):
        ost, omd, obd = O.block_verify(out[i], pks, stakes, 0)
        assert int(st[i]) == ost, i
        if ost != O.BLOCK_PARSE_ERROR:
            assert md[i].tobytes() == omd and bd[i].tobytes() == obd, i
    assert len({int(s) for s in st}) >= 3


def test_statement_kinds_and_ragged_lengths(engine, host_engine):
    """Every statement kind, shares of 0..700 bytes (pre-images 41 B .. ~9 KB), failures mixed in."""
    pks, stakes = small_committee()
    seeds = [B.authority_seed(a) for a in range(7)]
    prev = [B.genesis(a) for a in range(7)]
    rng = np.random.default_rng(5)
    out = []
    for r in range(1, 30):
        cur = []
        for a in range(7):
            k = int(rng.integers(1, 8))
            inc = [prev[a].reference()] + [prev[x].reference() for x in range(7) if x != a][: k - 1]
            loc = B.Locator(prev[(a + 1) % 7].reference(), int(rng.integers(0, 9)))
            sts = [("share", bytes(int(rng.integers(0, 700))))] * int(rng.integers(0, 3))
            sts += [("accept", loc), ("reject", loc, None), ("reject", loc, loc)][: int(rng.integers(0, 4))]
            sts += [("range", prev[(a + 2) % 7].reference(), 0, int(rng.integers(0, 5)))] * int(rng.integers(0, 9))
            cur.append(B.new_with_signer(a, r, inc, sts, r, bool(r & 1), 0, seeds[a], O.sign))
        out += [b.bincode() for b in cur]
        prev = cur
    out[3] = out[3][:-5] + bytes([out[3][-5] ^ 1]) + out[3][-4:]
    st, _, _ = agree(engine, host_engine, out, pks, stakes, 0)
    assert len({int(s) for s in st}) >= 3


def test_every_statement_and_metadata_byte_flipped(engine, host_engine):
    """One block holding every statement kind -- a Share, Vote Accept, Reject(None),
    Reject(Some(locator)) and a VoteRange -- with bit 0 and bit 7 of every byte from the statement
    count to the end flipped, one variant each: tags, vote options, the Some marker, both
    locators' digest lengths, the share length, the epoch marker and the signature length all
    change under some flip. Every form's verdict equals the host codec's, and the oracle's on
    every third variant (types.rs:315-376, data.rs:43-52)."""
    pks, stakes = small_committee()
    seeds = [B.authority_seed(a) for a in range(7)]
    prev = [B.genesis(a) for a in range(7)]
    inc = [prev[2].reference()] + [prev[x].reference() for x in range(7) if x != 2]  # own first, a quorum
    loc = B.Locator(prev[3].reference(), 4)
    sts = [("share", bytes(range(5))), ("accept", loc), ("reject", loc, None), ("reject", loc, loc),
           ("range", prev[4].reference(), 1, 3)]
    blk = B.new_with_signer(2, 1, inc, sts, 1, False, 0, seeds[2], O.sign).bincode()
    lo = 64 + 56 * len(inc)  # the statement count follows the header and the includes
    out = [blk]
    for i in range(lo, len(blk)):
        for bit in (0, 7):
            b = bytearray(blk)
            b[i] ^= 1 << bit
            out.append(bytes(b))
    st, md, bd = agree(engine, host_engine, out, pks, stakes, 0)
    assert int(st[0]) == 0
    for i in range(0, len(out), 3):
        ost, omd, obd = O.block_verify(out[i], pks, stakes, 0)
        assert int(st[i]) == ost, i
        if ost != O.BLOCK_PARSE_ERROR:
            assert md[i].tobytes() == omd and bd[i].tobytes() == obd, i
    assert (st == M.BLOCK_PARSE_ERROR).sum() > 20


def test_batch_path_through_device_ingest(engine, host_engine, golden):
    """>= MV_BATCH_MIN blocks: device parse feeds the batch equation; blocks rejected before
    the signature check stay out of it (no fallback without a bad signature)."""
    e = golden("block_edge.json")
    pks, stakes, epoch = committee(e["committee"])
    cases = [c for c in e["cases"] if not c["note"].startswith("bad signature")]
    reps = M.BATCH_MIN // len(cases) + 1
    bins = [bytes.fromhex(c["bincode"]) for c in cases] * reps
    b0, f0 = engine.batch_stats()
    st, _, _ = agree(engine, host_engine, bins, pks, stakes, epoch)
    b1, f1 = engine.batch_stats()
    assert [int(x) for x in st] == [c["status"] for c in cases] * reps
    assert b1 - b0 == 1 and f1 - f0 == 0


def test_device_resident_api(engine, golden):
    import torch

    g = golden("blocks_config4_sample.json")
    pks, stakes, epoch = committee(g["committee"])
    engine.set_committee(pks, stakes, epoch)
    bins = [b.bincode() for b in B.gen_config4(O.sign, rounds=2)]
    n = len(bins)
    lens = np.array([len(b) for b in bins], dtype=np.int64)
    offs = np.zeros(n, dtype=np.int64)
    offs[1:] = np.cumsum(lens)[:-1]  # packed back to back: unaligned block starts
    raw = np.frombuffer(b"".join(bins) + bytes(64), dtype=np.uint8)
    dev = torch.device("cuda", 0)
    d_buf = torch.from_numpy(raw.copy()).to(dev)
    d_off, d_len = torch.from_numpy(offs).to(dev), torch.from_numpy(lens).to(dev)
    d_st = torch.full((n,), 255, dtype=torch.uint8, device=dev)
    d_md = torch.zeros((n, 32), dtype=torch.uint8, device=dev)
    d_bd = torch.zeros((n, 32), dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    engine.dev_verify_blocks(0, d_buf, int(lens.sum()), d_off, d_len, d_st, d_md, d_bd)
    torch.cuda.synchronize()
    assert (d_st.cpu().numpy() == 0).all()
    assert hashlib.sha256(d_md.cpu().numpy().tobytes()).hexdigest() == g["sha256_msg_digests"]
    assert hashlib.sha256(d_bd.cpu().numpy().tobytes()).hexdigest() == g["sha256_block_digests"]


def test_blocks_beyond_the_lds_window(engine, host_engine):
    """Blocks whose bincode exceeds k_block_ingest's 10 KB LDS window take its one-lane
    path over global memory; mixed with window-sized blocks, corrupted and truncated ones."""
    pks, stakes = small_committee()
    seeds = [B.authority_seed(a) for a in range(7)]
    prev = [B.genesis(a) for a in range(7)]
    rng = np.random.default_rng(77)
    out = []
    for r in range(1, 5):
        cur = []
        for a in range(7):
            inc = [prev[a].reference()] + [prev[x].reference() for x in range(7) if x != a][:5]
            big = int(rng.integers(9000, 40000)) if (a + r) % 2 else int(rng.integers(0, 3000))
            sts = [("share", bytes(rng.integers(0, 256, size=big, dtype=np.uint8)))]
            sts += [("range", prev[(a + 2) % 7].reference(), 0, 3)] * 4
            cur.append(B.new_with_signer(a, r, inc, sts, r, False, 0, seeds[a], O.sign))
        out += [b.bincode() for b in cur]
        prev = cur
    big = [b for b in out if len(b) > 10240]
    assert len(big) >= 8
    bad = bytearray(big[0])
    bad[len(bad) // 2] ^= 4  # digest mismatch inside the share payload
    out += [bytes(bad), big[1][:-1], big[2][: len(big[2]) // 2]]
    st, md, bd = agree(engine, host_engine, out, pks, stakes, 0)
    for i in range(len(out)):
        ost, omd, obd = O.block_verify(out[i], pks, stakes, 0)
        assert int(st[i]) == ost, i
        if ost != O.BLOCK_PARSE_ERROR:
            assert md[i].tobytes() == omd and bd[i].tobytes() == obd, i
    assert int(st[-3]) == M.BLOCK_DIGEST_MISMATCH and int(st[-2]) == M.BLOCK_PARSE_ERROR
