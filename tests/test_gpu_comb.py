"""GPU: committee-key verification on per-key comb tables (comb.hip). Verdicts must equal the
golden fixtures, the oracle and the per-signature ladder (MV_FLAG_NO_COMB, k_verify) on the
same inputs, ZIP-215 edge cases included: small-order and non-canonical committee keys,
undecodable keys (MalformedPublicKey), s >= l, undecodable R."""
import numpy as np
import pytest

import mysticeti_amd as M
import oracle as O

pytestmark = pytest.mark.gpu


def arr(hexes, w):
    return np.frombuffer(b"".join(bytes.fromhex(h) for h in hexes), dtype=np.uint8).reshape(-1, w)


@pytest.fixture(scope="module")
def ladder():
    with M.Engine(devices=(0,), comb=False) as e:
        yield e


def test_zip215_corpus_as_committee(engine, ladder, golden):
    cases = [c for c in golden("zip215_corpus.json") if len(c["msg"]) == 64]
    keys = sorted({c["pk"] for c in cases})
    assert len(keys) <= 512
    kid = {k: i for i, k in enumerate(keys)}
    pks = arr(keys, 32)
    ok = engine.set_committee(pks, np.ones(len(keys), np.uint64))
    ok2 = ladder.set_committee(pks, np.ones(len(keys), np.uint64))
    assert (ok == ok2).all()
    for c in cases:  # key_ok: VerificationKey::try_from succeeds
        assert bool(ok[kid[c["pk"]]]) == O.point_decodes(bytes.fromhex(c["pk"])), c["note"]
    ki = np.array([kid[c["pk"]] for c in cases], np.uint32)
    msg, sig = arr([c["msg"] for c in cases], 32), arr([c["sig"] for c in cases], 64)
    st = engine.ed25519_verify(msg, sig, key_idx=ki)
    bad = [(c["note"], int(s), c["status"]) for c, s in zip(cases, st) if s != c["status"]]
    assert not bad, bad[:10]
    assert (ladder.ed25519_verify(msg, sig, key_idx=ki) == st).all()


def test_small_order_pairs_as_committee(engine, golden):
    """The 196 small-order (A, R) pairs with s = 0 accept for any message (cofactored check)."""
    cases = [c for c in golden("zip215_corpus.json") if c["note"].startswith("small-order A") and c["note"].endswith("s=0")]
    keys = sorted({c["pk"] for c in cases})
    kid = {k: i for i, k in enumerate(keys)}
    engine.set_committee(arr(keys, 32), np.ones(len(keys), np.uint64))
    ki = np.array([kid[c["pk"]] for c in cases], np.uint32)
    msg = np.tile(np.arange(32, dtype=np.uint8), (len(cases), 1))
    st = engine.ed25519_verify(msg, arr([c["sig"] for c in cases], 64), key_idx=ki)
    assert (st == 0).all()


def test_random_committee_vs_oracle_and_ladder(engine, ladder):
    rng = np.random.default_rng(31)
    na = 100
    seeds = rng.integers(0, 256, size=(na, 32), dtype=np.uint8)
    pks, _ = engine.ed25519_sign(seeds, np.zeros((na, 32), np.uint8))
    engine.set_committee(pks, np.ones(na, np.uint64))
    ladder.set_committee(pks, np.ones(na, np.uint64))
    n = 3000
    ki = rng.integers(0, na, size=n).astype(np.uint32)
    msg = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    _, sig = engine.ed25519_sign(seeds[ki], msg)
    sig = sig.copy()
    flip = rng.random(n) < 0.3
    pos = rng.integers(0, 512, size=n)
    for i in np.nonzero(flip)[0]:
        sig[i, pos[i] // 8] ^= 1 << (pos[i] % 8)
    l_bytes = (2**252 + 27742317777372353535851937790883648493).to_bytes(32, "little")
    sig[5, 32:] = np.frombuffer(l_bytes, np.uint8)  # s = l
    st = engine.ed25519_verify(msg, sig, key_idx=ki)
    ref = O.verify_batch(pks[ki], sig, msg)
    assert (st == ref).all()
    assert (ladder.ed25519_verify(msg, sig, key_idx=ki) == st).all()
    assert st[5] == 1 and (st != 0).sum() > n * 0.2


@pytest.mark.parametrize("n", [1, 2, 63, 64, 65, 127, 129, 1000])
def test_ragged_sizes(engine, n):
    rng = np.random.default_rng(100 + n)
    seeds = rng.integers(0, 256, size=(5, 32), dtype=np.uint8)
    pks, _ = engine.ed25519_sign(seeds, np.zeros((5, 32), np.uint8))
    engine.set_committee(pks, np.ones(5, np.uint64))
    ki = rng.integers(0, 5, size=n).astype(np.uint32)
    msg = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    _, sig = engine.ed25519_sign(seeds[ki], msg)
    assert (engine.ed25519_verify(msg, sig, key_idx=ki) == 0).all()
    sig = sig.copy()
    sig[n - 1, 0] ^= 1
    st = engine.ed25519_verify(msg, sig, key_idx=ki)
    assert st[n - 1] == 1 and (st[: n - 1] == 0).all()


def test_short_chain_and_one_lane_comb_kernels_agree(engine):
    """k_verify_comb16 (the online path: R decoded on a 16-lane row, table sums on quads) and
    k_verify_comb (one lane per signature)
    give identical verdicts on a committee batch with corrupted signatures, undecodable R,
    s >= l and an undecodable key, and both match the oracle."""
    rng = np.random.default_rng(47)
    na, n = 20, 300
    seeds = rng.integers(0, 256, size=(na, 32), dtype=np.uint8)
    pks, _ = engine.ed25519_sign(seeds, np.zeros((na, 32), np.uint8))
    pks = pks.copy()
    y = 2
    while O.point_decodes(y.to_bytes(32, "little")):
        y += 1
    pks[7] = np.frombuffer(y.to_bytes(32, "little"), np.uint8)  # does not decode: MalformedPublicKey
    engine.set_committee(pks, np.ones(na, np.uint64))
    ki = rng.integers(0, na, size=n).astype(np.uint32)
    msg = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    _, sig = engine.ed25519_sign(seeds[ki], msg)
    sig = sig.copy()
    sig[1::7, 40] ^= 4                  # corrupted s
    sig[2::11, 63] |= 0xF0              # s >= l
    sig[3::13, :32] = 0xFF              # R with y >= p (decodes or not, as ZIP-215 says)
    sig[5::17, 0] ^= 1                  # corrupted R
    out = {}
    for mode in ("0", "1"):
        with engine.option("MV_COMB_QUAD", int(mode)):
            out[mode] = engine.ed25519_verify(msg, sig, key_idx=ki)
    assert (out["0"] == out["1"]).all(), np.nonzero(out["0"] != out["1"])[0][:10]
    ref = O.verify_batch(pks[ki], sig, msg)
    assert (out["1"] == ref).all()
    assert (out["1"] == 0).sum() > n // 2 and (out["1"] == 2).any() and (out["1"] == 1).any()
