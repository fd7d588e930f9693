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


def test_concurrent_callers_are_coalesced(engine, opts):
    """16 threads each submit 1-4 blocks at a time (the per-peer tasks of net_sync.rs); every
    verdict and digest equals the serial call's, and the queue served the calls in fewer
    device passes than calls (the resident online service is off: every call queues)."""
    opts("MV_ONLINE", 0)
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


def _concurrent(engine, bins, threads=16, rounds=3, kmax=5):
    n = len(bins)
    got_st = np.full(n, 255, np.uint8)
    got_md = np.zeros((n, 32), np.uint8)
    got_bd = np.zeros((n, 32), np.uint8)
    errors = []

    def worker(t):
        rng = np.random.default_rng(100 + t)
        idx = list(range(t, n, threads))
        try:
            for _ in range(rounds):
                i = 0
                while i < len(idx):
                    k = int(rng.integers(1, kmax))
                    part = idx[i:i + k]
                    st, md, bd = engine.verify_blocks([bins[j] for j in part])
                    got_st[part], got_md[part], got_bd[part] = st, md, bd
                    i += k
        except Exception as e:  # pragma: no cover - reported below
            errors.append(e)

    th = [threading.Thread(target=worker, args=(t,)) for t in range(threads)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errors, errors
    return got_st, got_md, got_bd


def test_online_service_concurrent_callers(engine, opts):
    """The resident online service (k_online): 16 threads posting 1-4 blocks at a time get the
    verdicts and digests of the queue path (MV_ONLINE=0) and of the oracle; the service served
    the short-block calls (the long ones, > 2 KB per block, still queue)."""
    bins, pks, stakes = ragged_blocks(n_rounds=40, seed=13)
    engine.set_committee(pks, stakes, 0)
    opts("MV_ONLINE", 0)
    st_ref, md_ref, bd_ref = engine.verify_blocks(bins)
    opts("MV_ONLINE", 1)
    o0 = engine.online_stats()
    st, md, bd = _concurrent(engine, bins)
    o1 = engine.online_stats()
    assert (st == st_ref).all() and (md == md_ref).all() and (bd == bd_ref).all()
    assert o1[0] - o0[0] > 100 and o1[1] >= 1
    for i in range(0, len(bins), 37):
        ost, omd, obd = O.block_verify(bins[i], pks, stakes, 0)
        assert int(st[i]) == ost and md[i].tobytes() == omd and bd[i].tobytes() == obd, i


def test_online_service_edge_blocks_one_and_64_per_call(engine, golden, opts):
    """Every golden edge-case block through the service one per call and in 64-block calls
    (16 jobs of one request), against the fixture's verdicts and the queue path's digests."""
    fx = golden("block_edge.json")
    pks = np.array([bytes.fromhex(k) for k in fx["committee"]["pks"]], dtype=object)
    pks = np.frombuffer(b"".join(pks), dtype=np.uint8).reshape(-1, 32)
    stakes = np.array(fx["committee"]["stakes"], dtype=np.uint64)
    engine.set_committee(pks, stakes, fx["committee"]["epoch"])
    bins = [bytes.fromhex(c["bincode"]) for c in fx["cases"]]
    want = np.array([c["status"] for c in fx["cases"]], dtype=np.uint8)
    opts("MV_ONLINE", 0)
    _, md_ref, bd_ref = engine.verify_blocks(bins)
    opts("MV_ONLINE", 1)
    o0 = engine.online_stats()[0]
    one = [engine.verify_blocks([b]) for b in bins]
    st1 = np.array([r[0][0] for r in one], dtype=np.uint8)
    assert (st1 == want).all()
    for i, r in enumerate(one):
        assert (r[1][0] == md_ref[i]).all() and (r[2][0] == bd_ref[i]).all(), i
    reps = (bins * (64 // len(bins) + 1))[:64]
    st64, md64, bd64 = engine.verify_blocks(reps)
    w64 = (list(want) * (64 // len(bins) + 1))[:64]
    assert (st64 == np.array(w64, np.uint8)).all()
    assert engine.online_stats()[0] - o0 >= sum(1 for b in bins if len(b) < 1900)


def test_online_service_relaunches_after_idle_exit(engine, opts):
    """With a 300-us idle limit the kernel exits between calls 20 ms apart; the next call
    relaunches it and gets the right verdicts."""
    opts("MV_ONLINE_IDLE_US", 300)
    bins, pks, stakes = ragged_blocks(n_rounds=8, seed=3)
    engine.set_committee(pks, stakes, 0)  # stops a resident kernel (its idle limit was read at launch)
    short = [b for b in bins if len(b) < 1500][:6]
    l0 = engine.online_stats()[1]
    ref = [O.block_verify(b, pks, stakes, 0)[0] for b in short]
    import time

    for b, w in zip(short, ref):
        st, _, _ = engine.verify_blocks([b])
        assert int(st[0]) == w
        time.sleep(0.02)
    assert engine.online_stats()[1] - l0 >= len(short) - 1


def test_online_service_does_not_block_other_streams(engine, opts):
    """The resident kernel sits on a highest-priority stream (a queue of its own): while it is live (idle limit
    5 s here), a batch-path signature call and a queue-path block call on the engine's other
    streams complete at once, and the service is still the same launch afterwards."""
    import time

    opts("MV_ONLINE_IDLE_US", 5000000)
    bins, pks, stakes = ragged_blocks(n_rounds=8, seed=4)
    engine.set_committee(pks, stakes, 0)
    short = [b for b in bins if len(b) < 1500][:4]
    st, _, _ = engine.verify_blocks(short)  # launches the service
    l0 = engine.online_stats()[1]
    n = M.BATCH_MIN + 100
    rng = np.random.default_rng(8)
    seed = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    msg = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    t0 = time.perf_counter()
    pk, sig = engine.ed25519_sign(seed, msg)
    ss = engine.ed25519_verify(msg, sig, pk)
    opts("MV_ONLINE", 0)
    st_q, _, _ = engine.verify_blocks(short)
    opts("MV_ONLINE", 1)
    dt = time.perf_counter() - t0
    assert (ss == 0).all() and (st_q == st).all()
    assert dt < 2.0, dt  # not serialised behind the resident kernel's 5-s idle limit
    st2, _, _ = engine.verify_blocks(short)
    assert (st2 == st).all() and engine.online_stats()[1] == l0
    engine.set_committee(pks, stakes, 0)  # stops the service (no 5-s resident kernel left behind)


def test_online_service_size_limits_and_garbage(engine, opts):
    """The service takes calls of <= 64 blocks and <= 128 KB (long blocks included); 65 blocks
    go through the queue (as do long blocks under MV_ONLINE_LONG=0). Truncated, garbage and
    empty-length blocks give the queue path's verdicts (PARSE_ERROR, zero digests) either way."""
    bins, pks, stakes = ragged_blocks(n_rounds=20, seed=21)
    engine.set_committee(pks, stakes, 0)
    short = [b for b in bins if len(b) < 1200]
    rng = np.random.default_rng(5)
    calls = [short[:64], short[:65], short[:1], [bins[0][:10]] + short[:3], [bytes(8)] + short[:2],
             [rng.integers(0, 256, size=300, dtype=np.uint8).tobytes()] + short[5:9],
             [b for b in bins if len(b) > 2500][:3] + short[:1]]
    opts("MV_ONLINE", 0)
    want = [engine.verify_blocks(c) for c in calls]
    opts("MV_ONLINE", 1)
    for c, w in zip(calls, want):
        o0 = engine.online_stats()[0]
        got = engine.verify_blocks(c)
        took = engine.online_stats()[0] - o0
        for a, b in zip(got, w):
            assert (a == b).all()
        packed = sum((len(x) + 7) & ~7 for x in c)
        small_call = len(c) <= 64 and packed <= (128 << 10) and max(len(x) for x in c) + 32 <= 10240
        assert took == (1 if small_call else 0), (len(c), took)
    assert int(want[3][0][0]) == M.BLOCK_PARSE_ERROR and not want[3][1][0].any()


def test_online_service_long_blocks(engine, opts):
    """Config-4-shaped blocks (~9.5 KB, 66 VoteRanges, a 512-B share) take the service: one per
    call, and 12 in one call (< 128 KB), with a bad signature and a tampered digest among them;
    verdicts and both digests equal the queue path's and the oracle's."""
    import hashlib as H

    import mysticeti_amd.blocks as MB

    bins = list(MB.config4(engine, rounds=1))[:12]
    pks, stakes = MB.committee(engine, 100, distinct=True)
    engine.set_committee(pks, stakes, 0)
    b = bytearray(bins[3])  # an s bit: SIG_INVALID once the digest is recomputed
    b[-20] ^= 0x10
    b[24:56] = H.blake2b(M.block_preimage(bytes(b)) + bytes(b[-64:]), digest_size=32).digest()
    bins[3] = bytes(b)
    b = bytearray(bins[7])  # a stale claimed digest
    b[30] ^= 1
    bins[7] = bytes(b)
    calls = [bins[:1], bins[3:4], bins[7:8], bins]
    opts("MV_ONLINE", 0)
    want = [engine.verify_blocks(c) for c in calls]
    opts("MV_ONLINE", 1)
    for c, w in zip(calls, want):
        o0 = engine.online_stats()[0]
        got = engine.verify_blocks(c)
        assert engine.online_stats()[0] - o0 == 1
        for x, y in zip(got, w):
            assert (x == y).all()
    st, md, bd = want[-1]
    for i in (0, 3, 7, 11):
        ost, omd, obd = O.block_verify(bins[i], pks, stakes, 0)
        assert int(st[i]) == ost and md[i].tobytes() == omd and bd[i].tobytes() == obd, i
    assert int(st[3]) == 6 and int(st[7]) != 0


def test_online_service_survives_committee_changes(engine):
    """Callers keep posting through the service while the committee is set again (the resident
    kernel is stopped, the tables rebuilt, the next call relaunches it): no call hangs or fails,
    and every verdict is the oracle's."""
    import time

    bins, pks, stakes = ragged_blocks(n_rounds=10, seed=22)
    short = [b for b in bins if len(b) < 1200][:40]
    engine.set_committee(pks, stakes, 0)
    ref = [O.block_verify(b, pks, stakes, 0)[0] for b in short]
    errors, stop = [], [False]

    def worker(t):
        try:
            k = t
            while not stop[0]:
                st, _, _ = engine.verify_blocks([short[k % len(short)]])
                assert int(st[0]) == ref[k % len(short)]
                k += 7
        except Exception as e:  # pragma: no cover - reported below
            errors.append(e)

    th = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
    for x in th:
        x.start()
    l0 = engine.online_stats()[1]
    for _ in range(3):
        time.sleep(0.05)
        engine.set_committee(pks, stakes, 0)
    time.sleep(0.05)
    stop[0] = True
    for x in th:
        x.join(timeout=60)
    assert not any(x.is_alive() for x in th), "a caller hung"
    assert not errors, errors
    assert engine.online_stats()[1] - l0 >= 3  # relaunched after each stop


def test_online_service_launch_failure_fails_over_to_the_queue(opts):
    """A launch that fails after a request number was taken (fault injection, MV_ONLINE_INJECT)
    marks the service failed: that call returns MV_E_HIP, no caller hangs on the ring, and every
    later call -- 8 threads at once included -- is served by the submission queue with the
    oracle's verdicts (a failed request used to leave the ring stuck)."""
    bins, pks, stakes = ragged_blocks(n_rounds=8, seed=31)
    short = [b for b in bins if len(b) < 1200][:16]
    ref = [O.block_verify(b, pks, stakes, 0)[0] for b in short]
    with M.Engine(devices=(0,)) as eng:
        eng.set_committee(pks, stakes, 0)
        opts("MV_ONLINE_INJECT", 1, eng)
        with pytest.raises(M.MvError, match="injected"):
            eng.verify_blocks(short[:1])
        out = [None] * 8

        def worker(t):
            out[t] = [int(eng.verify_blocks([short[i]])[0][0]) for i in range(t, len(short), 8)]

        th = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
        for x in th:
            x.start()
        for x in th:
            x.join(timeout=60)
        assert not any(x.is_alive() for x in th)
        for t in range(8):
            assert out[t] == [ref[i] for i in range(t, len(short), 8)]
        assert eng.queue_stats()[0] >= len(short)


def test_buffer_growth_does_not_wait_for_the_live_service(opts):
    """While the resident kernel is live (5-s idle limit), calls that grow the engine's scratch
    -- a larger batch-path verify and a larger queue-path block call than the context has seen
    -- retire the old buffers instead of freeing them (hipFree drains the whole device, the
    resident kernel with it) and finish at once."""
    import time

    bins, pks, stakes = ragged_blocks(n_rounds=8, seed=32)
    short = [b for b in bins if len(b) < 1500][:4]
    rng = np.random.default_rng(9)
    n_small, n_big = M.BATCH_MIN + 7, 4 * M.BATCH_MIN + 11
    seed = rng.integers(0, 256, size=(n_big, 32), dtype=np.uint8)
    msg = rng.integers(0, 256, size=(n_big, 32), dtype=np.uint8)
    with M.Engine(devices=(0,)) as eng:
        pk, sig = eng.ed25519_sign(seed, msg)
        eng.set_committee(pks, stakes, 0)
        opts("MV_ONLINE_IDLE_US", 5000000, eng)
        # the scratch at its first sizes (before the service is live)
        assert (eng.ed25519_verify(msg[:n_small], sig[:n_small], pk[:n_small]) == 0).all()
        with eng.option("MV_ONLINE", 0):
            eng.verify_blocks(bins[:8])
        eng.verify_blocks(short)  # the service is live now
        l0 = eng.online_stats()[1]
        t0 = time.perf_counter()
        ss = eng.ed25519_verify(msg, sig, pk)  # grows the batch scratch
        with eng.option("MV_ONLINE", 0):
            sb, _, _ = eng.verify_blocks(bins * 3)  # grows the block scratch
        dt = time.perf_counter() - t0
        assert (ss == 0).all()
        big = bins * 3
        for i in range(0, len(big), 29):
            assert int(sb[i]) == O.block_verify(big[i], pks, stakes, 0)[0]
        assert dt < 2.0, dt
        eng.verify_blocks(short)
        assert eng.online_stats()[1] == l0  # the same launch served it


def test_retired_buffers_stay_bounded_over_growing_calls():
    """Calls of increasing size on the device API (three alternating streams, the bench's shape)
    grow the scratch rings many times; the retired buffers are freed once the slots' last calls
    are done (no resident kernel here), and growth is geometric, so the device memory held
    stays within a small factor of what one call at the final size needs (before,
    every growth kept the old allocation until mv_destroy)."""
    import torch

    dev = torch.device("cuda", 0)
    n_max = 1 << 19
    rng = np.random.default_rng(12)
    seed = torch.from_numpy(rng.integers(0, 256, size=(n_max, 32), dtype=np.uint8)).to(dev)
    msg = torch.from_numpy(rng.integers(0, 256, size=(n_max, 32), dtype=np.uint8)).to(dev)
    pk = torch.empty((n_max, 32), dtype=torch.uint8, device=dev)
    sig = torch.empty((n_max, 64), dtype=torch.uint8, device=dev)
    st = torch.empty((n_max,), dtype=torch.uint8, device=dev)
    ok = torch.zeros(1, dtype=torch.int32, device=dev)
    streams = [torch.cuda.Stream(dev) for _ in range(3)]

    def used():
        torch.cuda.synchronize()
        free, total = torch.cuda.mem_get_info(dev)
        return total - free

    def calls(eng, sizes):
        for k, n in enumerate(sizes):
            eng.dev_verify_batch(0, msg[:n], sig[:n], pk[:n], st[:n], ok, streams[k % 3].cuda_stream)
        torch.cuda.synchronize()

    with M.Engine(devices=(0,)) as eng:
        eng.dev_sign(0, seed, msg, pk, sig, streams[0].cuda_stream)
        torch.cuda.synchronize()
        base = used()
        calls(eng, [n_max] * 3)  # one call per slot at the final size
        ref = used() - base
        assert (st.cpu().numpy() == 0).all()
    with M.Engine(devices=(0,)) as eng:
        base = used()
        sizes = [min(n_max, (int(8192 * 1.3 ** k) + 1023) & ~1023) for k in range(17)]
        calls(eng, sizes + [n_max] * 3)  # (calls() ends in a device synchronize)
        calls(eng, [n_max])  # a call after it: every retiree's slot is done, so it frees them all
        grown = used() - base
        assert (st.cpu().numpy() == 0).all()
    # without freeing the retirees the held memory is ~3-4x ref
    assert grown <= 1.75 * ref + (64 << 20), (grown / 2**20, ref / 2**20)


def test_context_with_online_service_is_destroyed_and_the_process_exits():
    """The driver's smoke shape in a fresh process: mv_create, one call through the resident
    service, mv_destroy, interpreter exit -- within a time limit, several times over (round 4's
    driver smoke stalled after its last call)."""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = (
        "import sys; sys.path.insert(0, %r); sys.path.insert(0, %r)\n"
        "import numpy as np, blocks as B, oracle as O, mysticeti_amd as M\n"
        "blks = B.gen_config1(O.sign, rounds=2)\n"
        "pks = np.frombuffer(O.public_key(bytes(32)) * 4, dtype=np.uint8).reshape(4, 32)\n"
        "with M.Engine(devices=(0,)) as eng:\n"
        "    eng.set_committee(pks, np.ones(4, dtype=np.uint64), 0)\n"
        "    st, _, _ = eng.verify_blocks([b.bincode() for b in blks])\n"
        "    assert (st == 0).all() and eng.online_stats()[0] == 1\n"
        "print('destroyed', flush=True)\n" % (root, os.path.join(root, "oracle")))
    for rep in range(3):
        p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=90)
        assert p.returncode == 0 and "destroyed" in p.stdout, (rep, p.returncode, p.stdout[-500:], p.stderr[-2000:])


@pytest.mark.parametrize("kmax", [2, 5])
def test_online_service_one_block_callers(engine, golden, opts, kmax):
    """16 threads posting one block (kmax 2) or 1-4 blocks (kmax 5) at a time through the
    resident service, and every golden edge case one per call from 8 threads at once: the
    queue path's verdicts and digests, and the fixture's statuses."""
    bins, pks, stakes = ragged_blocks(n_rounds=40, seed=17)
    engine.set_committee(pks, stakes, 0)
    opts("MV_ONLINE", 0)
    st_ref, md_ref, bd_ref = engine.verify_blocks(bins)
    opts("MV_ONLINE", 1)
    st, md, bd = _concurrent(engine, bins, kmax=kmax)
    assert (st == st_ref).all() and (md == md_ref).all() and (bd == bd_ref).all()
    fx = golden("block_edge.json")
    epks = np.frombuffer(b"".join(bytes.fromhex(k) for k in fx["committee"]["pks"]), dtype=np.uint8).reshape(-1, 32)
    engine.set_committee(epks, np.array(fx["committee"]["stakes"], dtype=np.uint64), fx["committee"]["epoch"])
    ebins = [bytes.fromhex(c["bincode"]) for c in fx["cases"]] * 4
    want = np.array([c["status"] for c in fx["cases"]] * 4, dtype=np.uint8)
    est, _, _ = _concurrent(engine, ebins, threads=8, rounds=1, kmax=2)
    assert (est == want).all(), np.nonzero(est != want)[0][:8]
    engine.set_committee(pks, stakes, 0)
