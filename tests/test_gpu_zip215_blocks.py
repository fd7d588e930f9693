"""GPU: ZIP-215 signature edge cases inside whole StatementBlocks (tests/golden/block_zip215.json,
made by oracle/gen_fixtures.py and pinned to the pure-Python predicate and the C oracle).

crypto.rs:174-189 (msg = Blake2b-256(pre-image), then VerificationKey::verify) and
types.rs:346-348 (any signature error -> InvalidSignature): every block passes the other
checks, so its status is decided by the signature alone. The blocks go through every device
form that verifies a block signature:
  * the resident online service one block per call (the speculative R decode: workgroups of
    <= 3 blocks), 3 and 4 per call (4: the parse-then-decode workgroup) and 64 per call;
  * the submission queue (MV_FLAG_NO_ONLINE engine: one k_verify_comb16 pass);
  * the batch block path, tiled past MV_BATCH_MIN (the batch equation over committee keys,
    exact fallback for failing groups), on host buffers and on device buffers.
Every status and both digests must equal the fixture."""
import numpy as np
import pytest

import mysticeti_amd as M
import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def fx(golden):
    d = golden("block_zip215.json")
    pks = np.frombuffer(b"".join(bytes.fromhex(k) for k in d["committee"]["pks"]), dtype=np.uint8).reshape(-1, 32)
    stakes = np.array(d["committee"]["stakes"], dtype=np.uint64)
    bins = [bytes.fromhex(c["bincode"]) for c in d["cases"]]
    st = np.array([c["status"] for c in d["cases"]], dtype=np.uint8)
    md = np.array([np.frombuffer(bytes.fromhex(c["msg_digest"]), np.uint8) for c in d["cases"]])
    bd = np.array([np.frombuffer(bytes.fromhex(c["block_digest"]), np.uint8) for c in d["cases"]])
    notes = [c["note"] for c in d["cases"]]
    return pks, stakes, bins, st, md, bd, notes


def check(fx, idx, st, md, bd, what):
    _, _, _, w_st, w_md, w_bd, notes = fx
    for j, i in enumerate(idx):
        assert int(st[j]) == int(w_st[i]), f"{what}: case {i} ({notes[i]}): status {st[j]} != {w_st[i]}"
        assert (md[j] == w_md[i]).all() and (bd[j] == w_bd[i]).all(), f"{what}: case {i} ({notes[i]}): digest"


def test_fixture_matches_the_c_oracle(fx):
    pks, stakes, bins, w_st, w_md, w_bd, notes = fx
    assert (w_st == 0).sum() > 200 and (w_st == 6).sum() > 15  # both verdicts well represented
    for i, b in enumerate(bins):
        st, md, bd = O.block_verify(b, pks, stakes, 0)
        assert st == w_st[i] and md == w_md[i].tobytes() and bd == w_bd[i].tobytes(), notes[i]


@pytest.mark.parametrize("per_call", [1, 3, 4, 64])
def test_online_service(engine, fx, per_call):
    pks, stakes, bins, *_ = fx
    engine.set_committee(pks, stakes, 0)
    o0 = engine.online_stats()[0]
    n = len(bins)
    calls = 0
    for lo in range(0, n, per_call):
        idx = list(range(lo, min(n, lo + per_call)))
        st, md, bd = engine.verify_blocks([bins[i] for i in idx])
        check(fx, idx, st, md, bd, f"online, {per_call} per call")
        calls += 1
    assert engine.online_stats()[0] - o0 == calls  # every call took the resident service


def test_submission_queue(fx):
    pks, stakes, bins, *_ = fx
    with M.Engine(devices=(0,), online=False) as eng:
        eng.set_committee(pks, stakes, 0)
        st, md, bd = eng.verify_blocks(bins)
        check(fx, range(len(bins)), st, md, bd, "queue")
        assert eng.online_stats()[0] == 0


def test_batch_block_path(engine, fx):
    """The cases tiled (17 times, interleaved with their own order reversed) past
    MV_BATCH_MIN: one host call on the batch path, the equation over committee keys."""
    pks, stakes, bins, *_ = fx
    engine.set_committee(pks, stakes, 0)
    n = len(bins)
    idx = []
    for r in range(17):
        idx += list(range(n)) if r % 2 == 0 else list(range(n - 1, -1, -1))
    assert len(idx) >= M.BATCH_MIN
    b0 = engine.batch_stats()[0]
    st, md, bd = engine.verify_blocks([bins[i] for i in idx])
    check(fx, idx, st, md, bd, "batch path")
    assert engine.batch_stats()[0] > b0  # the batch equation ran


def test_batch_block_path_device_buffers(engine, fx):
    import torch

    pks, stakes, bins, *_ = fx
    engine.set_committee(pks, stakes, 0)
    n = len(bins)
    idx = [i % n for i in range(M.BATCH_MIN + 3 * n)]
    blobs = [bins[i] for i in idx]
    lens = np.array([len(b) for b in blobs], dtype=np.uint64)
    al = (lens + 7) & ~np.uint64(7)
    offs = np.zeros(len(blobs), dtype=np.uint64)
    offs[1:] = np.cumsum(al)[:-1]
    total = int(offs[-1] + al[-1]) + 16
    buf = np.zeros(total, dtype=np.uint8)
    for o, b in zip(offs, blobs):
        buf[int(o):int(o) + len(b)] = np.frombuffer(b, np.uint8)
    dev = torch.device("cuda:0")
    d_buf = torch.from_numpy(buf).to(dev)
    d_off = torch.from_numpy(offs.view(np.int64)).to(dev)
    d_len = torch.from_numpy(lens.view(np.int64)).to(dev)
    m = len(blobs)
    d_st = torch.zeros(m, dtype=torch.uint8, device=dev)
    d_md = torch.zeros((m, 32), dtype=torch.uint8, device=dev)
    d_bd = torch.zeros((m, 32), dtype=torch.uint8, device=dev)
    engine.dev_verify_blocks(0, d_buf, total - 16, d_off, d_len, d_st, d_md, d_bd)
    torch.cuda.synchronize()
    check(fx, idx, d_st.cpu().numpy(), d_md.cpu().numpy(), d_bd.cpu().numpy(), "batch path, device buffers")
