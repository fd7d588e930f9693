"""GPU: the batch path (batch.hip: one random linear combination checked as a
multi-scalar multiplication, exact per-signature fallback on the device).

Verdicts must equal the single-signature verdicts (oracle / golden fixtures) in every
case. The batch counters show which way each batch went: all-valid batches, including
ZIP-215 edge cases that single verification accepts (small-order and mixed-order A/R,
non-canonical encodings), must pass the combined equation without falling back;
batches with an invalid signature must fall back and still be exact.
"""
import numpy as np
import pytest

import mysticeti_amd as M
import oracle as O

pytestmark = pytest.mark.gpu


def arr(hexes, w):
    return np.frombuffer(b"".join(bytes.fromhex(h) for h in hexes), dtype=np.uint8).reshape(-1, w)


def signed(engine, n, seed):
    rng = np.random.default_rng(seed)
    s = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    m = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    pk, sig = engine.ed25519_sign(s, m)
    return m, sig, pk


def stats_delta(engine, fn):
    b0, f0 = engine.batch_stats()
    out = fn()
    b1, f1 = engine.batch_stats()
    return out, b1 - b0, f1 - f0


@pytest.mark.parametrize("n", [M.BATCH_MIN, M.BATCH_MIN + 1, 5000, 65536 + 17])
def test_valid_batches_pass_without_fallback(engine, n):
    msg, sig, pk = signed(engine, n, n)
    st, nb, nf = stats_delta(engine, lambda: engine.ed25519_verify(msg, sig, pk))
    assert (st == 0).all()
    assert nb == 1 and nf == 0


def test_one_bad_signature_falls_back_exactly(engine):
    n = 8192
    msg, sig, pk = signed(engine, n, 1)
    for where, byte in [(0, 33), (n - 1, 40), (4321, 50)]:  # s bytes: s stays < l, R decodes
        s2 = sig.copy()
        s2[where, byte] ^= 0x10
        st, nb, nf = stats_delta(engine, lambda: engine.ed25519_verify(msg, s2, pk))
        ref = O.verify_batch(pk, s2, msg)
        assert (st == ref).all()
        assert nb == 1 and nf == 1
        assert st[where] != 0 and (np.delete(st, where) == 0).all()


def test_wrong_message_falls_back(engine):
    n = 4096
    msg, sig, pk = signed(engine, n, 2)
    m2 = msg.copy()
    m2[77, 0] ^= 1
    st, nb, nf = stats_delta(engine, lambda: engine.ed25519_verify(m2, sig, pk))
    assert nf == 1 and st[77] == 1 and (np.delete(st, 77) == 0).all()


def test_prerejected_items_do_not_fail_the_batch(engine, golden):
    """s >= l, undecodable R and undecodable A are decided per signature before the
    combination and excluded from it: the batch still passes, the verdicts are exact."""
    n = 4096
    msg, sig, pk = signed(engine, n, 3)
    sig, pk = sig.copy(), pk.copy()
    l_bytes = (2**252 + 27742317777372353535851937790883648493).to_bytes(32, "little")
    sig[10, 32:] = np.frombuffer(l_bytes, np.uint8)  # s = l
    sig[11, 63] |= 0x80                              # s with bit 255
    cases = golden("zip215_corpus.json")
    bad_r = next(c for c in cases if c["status"] == 1 and c["note"].startswith("R undecodable"))
    bad_a = next(c for c in cases if c["status"] == 2)
    sig[12, :32] = np.frombuffer(bytes.fromhex(bad_r["sig"])[:32], np.uint8)
    pk[13] = np.frombuffer(bytes.fromhex(bad_a["pk"]), np.uint8)
    st, nb, nf = stats_delta(engine, lambda: engine.ed25519_verify(msg, sig, pk))
    ref = O.verify_batch(pk, sig, msg)
    assert (st == ref).all()
    assert list(st[10:14]) == [1, 1, 1, 2]
    assert nb == 1 and nf == 0


def test_zip215_accepts_pass_the_combination(engine, golden):
    """Every corpus case single verification accepts (small-order A and R, mixed-order
    points, non-canonical y, x = 0 with the sign bit) is also accepted by the combined
    cofactored equation: no fallback."""
    cases = [c for c in golden("zip215_corpus.json") if c["status"] == 0]
    assert len(cases) > 200
    # the small-order s = 0 pairs carry a 5-byte message in the corpus; their verdict
    # does not depend on the message (test_gpu_verify.test_zip215_small_order_msgs)
    m0 = arr([c["msg"] if len(c["msg"]) == 64 else "00" * 32 for c in cases], 32)
    s0, p0 = arr([c["sig"] for c in cases], 64), arr([c["pk"] for c in cases], 32)
    msg, sig, pk = signed(engine, M.BATCH_MIN, 4)
    msg, sig, pk = np.concatenate([m0, msg]), np.concatenate([s0, sig]), np.concatenate([p0, pk])
    st, nb, nf = stats_delta(engine, lambda: engine.ed25519_verify(msg, sig, pk))
    assert (st == 0).all()
    assert nb == 1 and nf == 0


def test_zip215_corpus_through_batch_path(engine, golden):
    cases = [c for c in golden("zip215_corpus.json") if len(c["msg"]) == 64]
    m0, s0, p0 = arr([c["msg"] for c in cases], 32), arr([c["sig"] for c in cases], 64), arr([c["pk"] for c in cases], 32)
    reps = M.BATCH_MIN // len(cases) + 1
    msg, sig, pk = np.tile(m0, (reps, 1)), np.tile(s0, (reps, 1)), np.tile(p0, (reps, 1))
    st, nb, nf = stats_delta(engine, lambda: engine.ed25519_verify(msg, sig, pk))
    want = np.tile(np.array([c["status"] for c in cases], np.uint8), reps)
    assert nb == 1
    assert (st == want).all()


def test_committee_key_index(engine):
    """key_idx rows (committee keys, the block path's layout) through the batch path."""
    rng = np.random.default_rng(5)
    seeds = rng.integers(0, 256, size=(7, 32), dtype=np.uint8)
    n = 6000
    ki = rng.integers(0, 7, size=n).astype(np.uint32)
    msg = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    pk, sig = engine.ed25519_sign(seeds[ki], msg)
    engine.set_committee(pk[[int(np.nonzero(ki == a)[0][0]) for a in range(7)]], np.ones(7, np.uint64))
    sig[99, 3] ^= 4
    st = engine.ed25519_verify(msg, sig, key_idx=ki)
    assert st[99] == 1 and (np.delete(st, 99) == 0).all()


def test_batch_and_single_paths_agree(golden):
    rng = np.random.default_rng(6)
    n = 4500
    with M.Engine(devices=(0,), batch=False) as single, M.Engine(devices=(0,)) as batched:
        msg, sig, pk = signed(single, n, 7)
        sig = sig.copy()
        bad = rng.random(n) < 0.002
        sig[bad, 33] ^= 2
        a = single.ed25519_verify(msg, sig, pk)
        b = batched.ed25519_verify(msg, sig, pk)
        assert (a == b).all() and (a[bad] == 1).all()
        assert single.batch_stats() == (0, 0) and batched.batch_stats() == (1, 1)


def test_device_api_flag(engine):
    import torch

    n = 8192
    msg, sig, pk = signed(engine, n, 8)
    dev = torch.device("cuda", 0)
    dm, ds, dp = (torch.from_numpy(x.copy()).to(dev) for x in (msg, sig, pk))
    dst = torch.full((n,), 255, dtype=torch.uint8, device=dev)
    ok = torch.zeros(1, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    engine.dev_verify_batch(0, dm, ds, dp, dst, ok)
    torch.cuda.synchronize()
    assert int(ok.item()) == 1 and (dst.cpu().numpy() == 0).all()
    ds[17, 50] ^= 1
    dst.fill_(255)
    torch.cuda.synchronize()
    engine.dev_verify_batch(0, dm, ds, dp, dst, ok)
    torch.cuda.synchronize()
    st = dst.cpu().numpy()
    assert int(ok.item()) == 0 and st[17] == 1 and (np.delete(st, 17) == 0).all()


def test_committee_keys_batch_equation_uses_comb_a(engine, golden):
    """With committee keys the batch path reads A from the comb tables of mv_set_committee
    (no per-signature A decode). The combined equation must still hold for valid rows and
    for the ZIP-215 edge-case keys (small-order, non-canonical), and a key that does not
    decode must give MalformedPublicKey (status 2) without failing the combination."""
    cases = [c for c in golden("zip215_corpus.json") if len(c["msg"]) == 64 and c["status"] in (0, 2)]
    rng = np.random.default_rng(11)
    seeds = rng.integers(0, 256, size=(7, 32), dtype=np.uint8)
    n = 6000
    ki = rng.integers(0, 7, size=n).astype(np.uint32)
    msg = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    pk, sig = engine.ed25519_sign(seeds[ki], msg)
    keys = [bytes(pk[int(np.nonzero(ki == a)[0][0])]) for a in range(7)]
    for c in cases:
        if bytes.fromhex(c["pk"]) not in keys:
            keys.append(bytes.fromhex(c["pk"]))
    assert len(keys) <= 512
    com = np.frombuffer(b"".join(keys), dtype=np.uint8).reshape(-1, 32)
    engine.set_committee(com, np.ones(len(keys), np.uint64))
    cki = np.array([keys.index(bytes.fromhex(c["pk"])) for c in cases], np.uint32)
    msg = np.concatenate([msg, arr([c["msg"] for c in cases], 32)])
    sig = np.concatenate([sig, arr([c["sig"] for c in cases], 64)])
    ki = np.concatenate([ki, cki])
    want = np.concatenate([np.zeros(n, np.uint8), np.array([c["status"] for c in cases], np.uint8)])
    st, nb, nf = stats_delta(engine, lambda: engine.ed25519_verify(msg, sig, key_idx=ki))
    assert nb == 1 and nf == 0
    assert (st == want).all()
    assert (want == 2).any()


def counters_delta(engine, fn):
    c0 = engine.batch_counters()
    out = fn()
    c1 = engine.batch_counters()
    return out, tuple(b - a for a, b in zip(c0, c1))


@pytest.mark.parametrize("n,groups,want_groups", [(16384, 8, 8), (16384 + 100, 8, 6), (9000, 16, 9)])
def test_sub_batch_equations_reverify_only_failing_groups(engine, n, groups, want_groups):
    """Fixed sub-batch equations: every group's equation holds on a valid batch; bad
    signatures fail exactly the groups that hold them, and only those are re-verified
    (the verdicts stay exact)."""
    msg, sig, pk = signed(engine, n, 21 + n)
    engine.set_batch_groups(groups)
    try:
        st, d = counters_delta(engine, lambda: engine.ed25519_verify(msg, sig, pk))
        assert (st == 0).all()
        assert d == (1, 0, want_groups, 0)
        gsize = -(-(-(-n // 1024)) // groups) * 1024  # whole 1024-signature chunks per group
        s2 = sig.copy()
        bad = [5, 3 * gsize + 7, 3 * gsize + 100, n - 1]
        for b in bad:
            s2[b, 40] ^= 0x10  # s stays < l, R decodes: only an equation can catch it
        st, d = counters_delta(engine, lambda: engine.ed25519_verify(msg, s2, pk))
        ref = O.verify_batch(pk, s2, msg)
        assert (st == ref).all() and (st[bad] == 1).all()
        failing = len({b // gsize for b in bad})
        assert d == (1, 1, want_groups, failing)
    finally:
        engine.set_batch_groups(0)


def test_adaptive_guard_after_a_failed_batch():
    """Default policy: one batch equation per batch; a failed equation arms the guard, and
    the next batches are cut into 8 (a bad signature then re-verifies one group)."""
    with M.Engine(devices=(0,)) as eng:
        n = 16384
        msg, sig, pk = signed(eng, n, 31)
        s2 = sig.copy()
        s2[100, 40] ^= 0x10
        st, d = counters_delta(eng, lambda: eng.ed25519_verify(msg, s2, pk))
        assert st[100] == 1 and (np.delete(st, 100) == 0).all()
        assert d == (1, 1, 1, 1)
        st, d = counters_delta(eng, lambda: eng.ed25519_verify(msg, s2, pk))
        assert st[100] == 1 and (np.delete(st, 100) == 0).all()
        assert d == (1, 1, 8, 1)
        st, d = counters_delta(eng, lambda: eng.ed25519_verify(msg, sig, pk))
        assert (st == 0).all() and d == (1, 0, 8, 0)
        eng.set_batch_groups(0)  # setting the policy clears the guard: one equation again
        st, d = counters_delta(eng, lambda: eng.ed25519_verify(msg, sig, pk))
        assert (st == 0).all() and d == (1, 0, 1, 0)


def routes_delta(engine, fn):
    r0 = engine.batch_routes()
    out = fn()
    r1 = engine.batch_routes()
    return out, tuple(b - a for a, b in zip(r0, r1))


def test_dense_failures_route_to_the_single_path_and_back():
    """Config 3 (~1% of the signatures bad): the first failed equation arms the guard; a guarded
    batch failing in every group sends the next batches straight to per-signature verification
    (no wasted MSM); a batch there with few invalid signatures sends the policy back to the
    (guarded) equation. Verdicts stay exact on every route (crypto.rs:188, net_sync.rs:352-361)."""
    with M.Engine(devices=(0,)) as eng:
        n = 16384
        msg, sig, pk = signed(eng, n, 33)
        rng = np.random.default_rng(34)
        bad = np.sort(rng.choice(n, n // 100, replace=False))
        s_bad = sig.copy()
        s_bad[bad, 40] ^= 0x10  # s stays < l, R decodes: only an equation or a single verify sees it
        want = np.zeros(n, np.uint8)
        want[bad] = 1
        run = lambda s: lambda: eng.ed25519_verify(msg, s, pk)
        st, d = routes_delta(eng, run(s_bad))  # one equation, failed: the guard is armed
        assert (st == want).all() and d == (1, 0, 0)
        st, d = routes_delta(eng, run(s_bad))  # 8 guarded equations, all failed: dense
        assert (st == want).all() and d == (1, 0, 1)
        st, d = routes_delta(eng, run(s_bad))  # straight to the single path
        assert (st == want).all() and d == (0, 1, 0)
        st, d = routes_delta(eng, run(s_bad))  # still dense: stays there
        assert (st == want).all() and d == (0, 1, 0)
        st, d = routes_delta(eng, run(sig))  # a clean batch on the single path ...
        assert (st == 0).all() and d == (0, 1, 0)
        st, d = counters_delta(eng, run(sig))  # ... sends the next one back to the guarded equation
        assert (st == 0).all() and d == (1, 0, 8, 0)
        st, d = routes_delta(eng, run(s_bad[:, :]))  # guarded, dense again: detected at once
        assert (st == want).all() and d == (1, 0, 1)
        eng.set_batch_groups(0)  # setting the policy clears the route too
        st, d = routes_delta(eng, run(sig))
        assert (st == 0).all() and d == (1, 0, 0)


def test_dense_route_on_device_buffers():
    """The same route through mv_dev_ed25519_verify_batch on three alternating streams (the
    bench's adversarial leg): exact statuses on every call, d_batch_ok 0 on single-path calls."""
    import torch

    with M.Engine(devices=(0,)) as eng:
        n = 8192
        msg, sig, pk = signed(eng, n, 35)
        bad = np.arange(7, n, 97)
        sig = sig.copy()
        sig[bad, 40] ^= 0x10
        want = np.zeros(n, np.uint8)
        want[bad] = 1
        dev = torch.device("cuda", 0)
        d_msg, d_sig, d_pk = (torch.from_numpy(x.copy()).to(dev) for x in (msg, sig, pk))
        streams = [torch.cuda.Stream(dev) for _ in range(3)]
        d_st = [torch.full((n,), 255, dtype=torch.uint8, device=dev) for _ in range(3)]
        d_ok = [torch.full((1,), 7, dtype=torch.int32, device=dev) for _ in range(3)]
        torch.cuda.synchronize()
        r0 = eng.batch_routes()
        for k in range(12):
            j = k % 3
            eng.dev_verify_batch(0, d_msg, d_sig, d_pk, d_st[j], d_ok[j], streams[j].cuda_stream)
            if j == 2:
                torch.cuda.synchronize()
                for x in d_st:
                    assert (x.cpu().numpy() == want).all()
                assert all(int(x.item()) == 0 for x in d_ok)
        d = [b - a for a, b in zip(r0, eng.batch_routes())]
        assert d[1] >= 6 and d[2] >= 1 and d[0] + d[1] == 12


@pytest.mark.parametrize("pinned", [False, True])
@pytest.mark.parametrize("committee", [False, True])
def test_pipelined_host_batches(engine, committee, pinned):
    """Large host-buffer calls, through the default direct path (pageable arrays) and through
    the chunked copy-beside-verify pipeline that pinned inputs (mv_host_alloc) take: ragged
    sizes, committee-key rows and bad signatures far apart keep exact verdicts."""
    rng = np.random.default_rng(41 + committee)
    n = 9 * M.BATCH_MIN + 333
    msg = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    if committee:
        seeds = rng.integers(0, 256, size=(9, 32), dtype=np.uint8)
        ki = rng.integers(0, 9, size=n).astype(np.uint32)
        pk, sig = engine.ed25519_sign(seeds[ki], msg)
        engine.set_committee(pk[[int(np.nonzero(ki == a)[0][0]) for a in range(9)]], np.ones(9, np.uint64))
    else:
        pk, sig = engine.ed25519_sign(rng.integers(0, 256, size=(n, 32), dtype=np.uint8), msg)
    sig = sig.copy()
    bad = [3, n // 3, n - 2]
    sig[bad, 45] ^= 0x20
    if pinned:
        def pin(a):
            h = engine.host_empty(a.shape, a.dtype)
            h[...] = a
            return h
        msg, sig, pk = pin(msg), pin(sig), pin(pk)
        if committee:
            ki = pin(ki)
    st = engine.ed25519_verify(msg, sig, key_idx=ki) if committee else engine.ed25519_verify(msg, sig, pk)
    assert (st[bad] == 1).all() and (np.delete(st, bad) == 0).all()


@pytest.mark.parametrize("committee", [False, True])
def test_streamed_pinned_inputs_many_batches(committee):
    """Pinned inputs with max_batch = 8,192: a call of 5 batches + a ragged tail on the
    chunked-copy streamed path (input buffers reused across batches, copy chunks gating
    k_bv_prep chunk by chunk), twice in a row, with bad signatures in the first, a middle and
    the last batch: exact verdicts, the same as pageable inputs."""
    rng = np.random.default_rng(77 + committee)
    n = 5 * 8192 + 77
    with M.Engine(devices=(0,), max_batch=8192) as eng:
        msg = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
        if committee:
            seeds = rng.integers(0, 256, size=(5, 32), dtype=np.uint8)
            ki = rng.integers(0, 5, size=n).astype(np.uint32)
            pk, sig = eng.ed25519_sign(seeds[ki], msg)
            eng.set_committee(pk[[int(np.nonzero(ki == a)[0][0]) for a in range(5)]], np.ones(5, np.uint64))
        else:
            pk, sig = eng.ed25519_sign(rng.integers(0, 256, size=(n, 32), dtype=np.uint8), msg)
        sig = sig.copy()
        bad = [0, 8191, 8192, 3 * 8192 + 5, n - 1]
        sig[bad, 40] ^= 0x10

        def pin(a):
            h = eng.host_empty(a.shape, a.dtype)
            h[...] = a
            return h

        pm, ps, pp = pin(msg), pin(sig), pin(pk)
        pki = pin(ki) if committee else None
        for _ in range(2):
            st = eng.ed25519_verify(pm, ps, key_idx=pki) if committee else eng.ed25519_verify(pm, ps, pp)
            assert (st[bad] == 1).all() and (np.delete(st, bad) == 0).all()
        st2 = eng.ed25519_verify(msg, sig, key_idx=ki) if committee else eng.ed25519_verify(msg, sig, pk)
        assert (st2 == st).all()


@pytest.mark.parametrize("committee", [False, True])
def test_two_concurrent_pinned_callers(committee):
    """Two threads calling mv_ed25519_verify on pinned inputs at once (the reference's one task
    per peer, net_sync.rs:214-221): the calls overlap (the enqueue holds the context, the wait
    for the verdicts does not), each with bad signatures of its own in every batch, several
    rounds: every verdict exact, the same as one caller alone."""
    import threading

    rng = np.random.default_rng(505 + committee)
    n = 9 * M.BATCH_MIN + 1111
    with M.Engine(devices=(0,)) as eng:
        data = []
        for c in range(2):
            msg = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
            if committee:
                seeds = rng.integers(0, 256, size=(6, 32), dtype=np.uint8)
                ki = rng.integers(0, 6, size=n).astype(np.uint32)
                pk, sig = eng.ed25519_sign(seeds[ki], msg)
                if c == 0:
                    com_seeds, com_pk = seeds, pk[[int(np.nonzero(ki == a)[0][0]) for a in range(6)]]
                else:  # both callers sign with the committee's keys
                    ki = rng.integers(0, 6, size=n).astype(np.uint32)
                    pk, sig = eng.ed25519_sign(com_seeds[ki], msg)
            else:
                ki = None
                pk, sig = eng.ed25519_sign(rng.integers(0, 256, size=(n, 32), dtype=np.uint8), msg)
            sig = sig.copy()
            bad = np.sort(rng.choice(n, 7, replace=False))
            sig[bad, 40] ^= 0x10
            want = np.zeros(n, np.uint8)
            want[bad] = 1

            def pin(a):
                h = eng.host_empty(a.shape, a.dtype)
                h[...] = a
                return h

            data.append((pin(msg), pin(sig), pin(pk), pin(ki) if committee else None, want))
        if committee:
            eng.set_committee(com_pk, np.ones(6, np.uint64))
        got = [[], []]
        errors = []

        def caller(c):
            pm, ps, pp, pki, _ = data[c]
            try:
                for _ in range(4):
                    st = eng.ed25519_verify(pm, ps, key_idx=pki) if committee else eng.ed25519_verify(pm, ps, pp)
                    got[c].append(st.copy())
            except Exception as e:  # pragma: no cover - reported below
                errors.append(e)

        th = [threading.Thread(target=caller, args=(c,)) for c in range(2)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        assert not errors, errors
        for c in range(2):
            assert len(got[c]) == 4
            for st in got[c]:
                assert (st == data[c][4]).all(), np.nonzero(st != data[c][4])[0][:8]


@pytest.mark.parametrize("bal", [0, 1, 7, 200])
@pytest.mark.parametrize("groups", [0, 5])
def test_bucket_forms_agree(engine, opts, bal, groups):
    """Both bucket kernels (one lane per bucket: MV_BUCKET_BAL=0; equal entries per lane: 1 =
    64 per lane, or 7 / 200 entries so that lanes split buckets many ways or hold many
    buckets) give equations that hold on valid batches and fail exactly where a signature is
    bad, with and without sub-batch equations."""
    opts("MV_BUCKET_BAL", bal)
    n = 9000
    msg, sig, pk = signed(engine, n, 77)
    engine.set_batch_groups(groups)
    try:
        st, nb, nf = stats_delta(engine, lambda: engine.ed25519_verify(msg, sig, pk))
        assert (st == 0).all() and nb == 1 and nf == 0
        s2 = sig.copy()
        s2[[3, 4444, n - 1], 40] ^= 0x10
        st, nb, nf = stats_delta(engine, lambda: engine.ed25519_verify(msg, s2, pk))
        assert (st == O.verify_batch(pk, s2, msg)).all() and nb == 1 and nf == 1
    finally:
        engine.set_batch_groups(0)


@pytest.mark.parametrize("bal", [1, 0])
def test_streamed_small_copy_chunks(engine, opts, bal):
    """Pinned inputs in 4,096-signature copy chunks (MV_STREAM_CHUNK_LOG2=12: k_bv_prep runs
    chunk by chunk as the copies land), with both bucket kernels: the equation holds on a valid
    call without a fallback, and bad signatures at chunk edges come back exact."""
    for name, v in (("MV_STREAM_CHUNK_LOG2", 12), ("MV_BUCKET_BAL", bal)):
        opts(name, v)
    n = 9 * M.BATCH_MIN + 333
    msg, sig, pk = signed(engine, n, 91 + bal)

    def pin(a):
        h = engine.host_empty(a.shape, a.dtype)
        h[...] = a
        return h

    engine.set_batch_groups(1)  # one equation per batch (no adaptive guard from earlier tests)
    try:
        pm, ps, pp = pin(msg), pin(sig), pin(pk)
        st, nb, nf = stats_delta(engine, lambda: engine.ed25519_verify(pm, ps, pp))
        assert (st == 0).all() and nf == 0
        bad = [0, 4095, 4096, n // 2, n - 1]
        ps[bad, 40] ^= 0x10
        st = engine.ed25519_verify(pm, ps, pp)
        assert (st[bad] == 1).all() and (np.delete(st, bad) == 0).all()
    finally:
        engine.set_batch_groups(0)


@pytest.mark.parametrize("rows", [1, 0])
@pytest.mark.parametrize("groups", [0, 3])
def test_final_forms_agree(engine, opts, rows, groups):
    """k_bv_final's Horner with one DPP row per coordinate (MV_FINAL_ROWS=1, one equation) and
    with four lanes per point (0, or several sub-batch equations): valid batches hold without a
    fallback (a wrong window sum, doubling or addition would fail the equation), and a bad
    signature fails exactly its group."""
    opts("MV_FINAL_ROWS", rows)
    n = 6000
    msg, sig, pk = signed(engine, n, 303)
    engine.set_batch_groups(groups)
    try:
        st, nb, nf = stats_delta(engine, lambda: engine.ed25519_verify(msg, sig, pk))
        assert (st == 0).all() and nb == 1 and nf == 0
        s2 = sig.copy()
        s2[[17, n - 5], 40] ^= 0x10
        st, nb, nf = stats_delta(engine, lambda: engine.ed25519_verify(msg, s2, pk))
        assert (st == O.verify_batch(pk, s2, msg)).all() and nb == 1 and nf == 1
    finally:
        engine.set_batch_groups(0)
