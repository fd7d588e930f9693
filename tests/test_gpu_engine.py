"""GPU: the engine around the kernels -- the block submission queue (concurrent callers of
mv_verify_blocks merged into shared device passes, net_sync.rs:214-221 / 314-386) and the
multi-device sharding (contiguous shards balanced by bytes, verdicts written back per item),
exercised on one GPU through logical shards (mv_config.shards_per_device)."""
import threading

import numpy as np
import pytest

import blocks as B
import mysticeti_amd as M
import oracle as O

pytestmark = pytest.mark.gpu


def ragged_blocks(n_rounds=30, seed=5):
    seeds = [B.authority_seed(a) for a in range(7)]
    pks = np.frombuffer(b"".join(O.public_key(s) for s in seeds), dtype=np.uint8).reshape(-1, 32)
    stakes = np.array([3, 1, 1, 2, 1, 1, 1], dtype=np.uint64)
    prev = [B.genesis(a) for a in range(7)]
    blocks = []
    rng = np.random.default_rng(seed)
    for r in range(1, n_rounds + 1):
        for a in range(7):
            k = int(rng.integers(1, 8))
            inc = [prev[a].reference()] + [prev[x].reference() for x in range(7) if x != a][: k - 1]
            sts = [("share", bytes(int(rng.integers(0, 3000))))] * int(rng.integers(0, 3))
            sts += [("range", prev[(a + 1) % 7].reference(), 0, int(rng.integers(0, 5)))] * int(rng.integers(0, 20))
            blocks.append(B.new_with_signer(a, r, inc, sts, r, False, 0, seeds[a], O.sign))
        prev = blocks[-7:]
    bins = [b.bincode() for b in blocks]
    bins[3] = bins[3][:-5] + bytes([bins[3][-5] ^ 1]) + bins[3][-4:]  # bad signature
    bins[10] = bins[10][:60]                                           # truncated
    t = bytearray(bins[50])
    t[-20] ^= 4                                                        # tampered: stale digest
    bins[50] = bytes(t)
    return bins, pks, stakes


@pytest.mark.parametrize("shards", [2, 3])
def test_logical_shards_match_one_device(engine, shards):
    bins, pks, stakes = ragged_blocks()
    engine.set_committee(pks, stakes, 0)
    st1, md1, bd1 = engine.verify_blocks(bins)
    with M.Engine(devices=(0,), shards_per_device=shards) as es:
        es.set_committee(pks, stakes, 0)
        st, md, bd = es.verify_blocks(bins)
        assert (st == st1).all() and (md == md1).all() and (bd == bd1).all()
        # signatures: count-balanced shards, each >= MV_BATCH_MIN takes the batch path
        n = shards * M.BATCH_MIN + 77
        rng = np.random.default_rng(shards)
        seed = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
        msg = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
        pk, sig = es.ed25519_sign(seed, msg)
        sig[[0, n // 2, n - 1], 40] ^= 0x10
        ss = es.ed25519_verify(msg, sig, pk)
        assert (ss == O.verify_batch(pk, sig, msg)).all()
        assert es.batch_stats()[0] == shards
    for i, b in enumerate(bins):
        ost, omd, obd = O.block_verify(b, pks, stakes, 0)
        assert int(st1[i]) == ost, i


def test_concurrent_callers_are_coalesced(engine):
    """16 threads each submit 1-4 blocks at a time (the per-peer tasks of net_sync.rs); every
    verdict and digest equals the serial call's, and the queue served the calls in fewer
    device passes than calls."""
    bins, pks, stakes = ragged_blocks(n_rounds=40, seed=9)
    engine.set_committee(pks, stakes, 0)
    st_ref, md_ref, bd_ref = engine.verify_blocks(bins)
    n = len(bins)
    got_st = np.full(n, 255, np.uint8)
    got_md = np.zeros((n, 32), np.uint8)
    got_bd = np.zeros((n, 32), np.uint8)
    errors = []
    c0 = engine.queue_stats()

    def worker(t):
        rng = np.random.default_rng(100 + t)
        idx = list(range(t, n, 16))
        try:
            for _ in range(3):
                i = 0
                while i < len(idx):
                    k = int(rng.integers(1, 5))
                    part = idx[i:i + k]
                    st, md, bd = engine.verify_blocks([bins[j] for j in part])
                    got_st[part], got_md[part], got_bd[part] = st, md, bd
                    i += k
        except Exception as e:  # pragma: no cover - reported below
            errors.append(e)

    th = [threading.Thread(target=worker, args=(t,)) for t in range(16)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errors, errors
    c1 = engine.queue_stats()
    calls, passes = c1[0] - c0[0], c1[1] - c0[1]
    assert (got_st == st_ref).all() and (got_md == md_ref).all() and (got_bd == bd_ref).all()
    assert len({int(s) for s in st_ref}) >= 3
    assert calls >= 16 * 3 * (n // 16) // 4 and passes < calls
