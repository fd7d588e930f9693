"""GPU: ZIP-215 verification and RFC 8032 signing through the C ABI, bit-exact vs the
golden fixtures and the oracle (configs 2 and 3 of BASELINE.json at full 1M size)."""
import hashlib
import struct

import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu


def arr(hexes, w):
    return np.frombuffer(b"".join(bytes.fromhex(h) for h in hexes), dtype=np.uint8).reshape(-1, w)


def test_sig_kats(engine, golden):
    cases = golden("sig_kat.json")
    seed, msg = arr([c["seed"] for c in cases], 32), arr([c["msg"] for c in cases], 32)
    pk, sig = arr([c["pk"] for c in cases], 32), arr([c["sig"] for c in cases], 64)
    assert (engine.ed25519_verify(msg, sig, pk) == 0).all()
    gpk, gsig = engine.ed25519_sign(seed, msg)
    assert (gpk == pk).all() and (gsig == sig).all()


def test_zip215_corpus(engine, golden):
    cases = [c for c in golden("zip215_corpus.json") if len(c["msg"]) == 64]
    st = engine.ed25519_verify(arr([c["msg"] for c in cases], 32), arr([c["sig"] for c in cases], 64),
                               arr([c["pk"] for c in cases], 32))
    bad = [(c["note"], int(s), c["status"]) for c, s in zip(cases, st) if s != c["status"]]
    assert not bad, bad[:10]


def test_zip215_small_order_msgs(engine, golden):
    """The 196 small-order (A, R) pairs use a 5-byte message in the corpus; re-check with 32-byte messages
    against the C oracle (verdict does not depend on the message for s = 0 small-order pairs)."""
    cases = [c for c in golden("zip215_corpus.json") if c["note"].startswith("small-order A") and c["note"].endswith("s=0")]
    pk, sig = arr([c["pk"] for c in cases], 32), arr([c["sig"] for c in cases], 64)
    msg = np.tile(np.arange(32, dtype=np.uint8), (len(cases), 1))
    st = engine.ed25519_verify(msg, sig, pk)
    ref = O.verify_batch(pk, sig, msg)
    assert (st == ref).all() and (st == 0).all()


def test_random_corruptions_vs_oracle(engine):
    rng = np.random.default_rng(11)
    n = 4096
    seed = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    msg = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    pk, sig = O.sign_batch(seed, msg)
    sig = sig.copy()
    flip = rng.random(n) < 0.3
    pos = rng.integers(0, 512, size=n)
    for i in np.nonzero(flip)[0]:
        sig[i, pos[i] // 8] ^= 1 << (pos[i] % 8)
    msg2 = msg.copy()
    mflip = rng.random(n) < 0.05
    msg2[mflip, 0] ^= 0x80
    st = engine.ed25519_verify(msg2, sig, pk)
    ref = O.verify_batch(pk, sig, msg2)
    assert (st == ref).all()
    assert (st != 0).sum() > n * 0.2


def test_ragged_batch_sizes(engine):
    rng = np.random.default_rng(12)
    for n in [1, 2, 63, 64, 65, 255, 257, 1000]:
        seed = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
        msg = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
        pk, sig = engine.ed25519_sign(seed, msg)
        opk, osig = O.sign_batch(seed, msg)
        assert (pk == opk).all() and (sig == osig).all(), n
        assert (engine.ed25519_verify(msg, sig, pk) == 0).all(), n
    st = engine.ed25519_verify(np.zeros((0, 32), np.uint8), np.zeros((0, 64), np.uint8), np.zeros((0, 32), np.uint8))
    assert st.shape == (0,)


def corpus(n):
    seed = np.frombuffer(b"".join(hashlib.sha512(b"mysti-seed" + struct.pack("<Q", i)).digest()[:32]
                                  for i in range(n)), dtype=np.uint8).reshape(n, 32)
    msg = np.frombuffer(b"".join(hashlib.blake2b(b"mysti-msg" + struct.pack("<Q", i), digest_size=32).digest()
                                 for i in range(n)), dtype=np.uint8).reshape(n, 32)
    return seed, msg


@pytest.mark.slow
def test_config2_and_config3_1m(engine, golden):
    g2, g3 = golden("batch_config2.json"), golden("batch_config3.json")
    n = g2["n"]
    seed, msg = corpus(n)
    assert hashlib.sha256(msg.tobytes()).hexdigest() == g2["sha256_msg"]
    pk, sig = engine.ed25519_sign(seed, msg)
    assert hashlib.sha256(pk.tobytes()).hexdigest() == g2["sha256_pk"]
    assert hashlib.sha256(sig.tobytes()).hexdigest() == g2["sha256_sig"]
    st = engine.ed25519_verify(msg, sig, pk)
    assert hashlib.sha256(st.tobytes()).hexdigest() == g2["sha256_status"]
    assert int((st == 0).sum()) == g2["accepted"]
    # config 3: 1% single-bit corruptions of R || s
    sigc = sig.copy()
    for i in range(n):
        c = hashlib.sha256(b"mysti-corrupt" + struct.pack("<Q", i)).digest()
        if int.from_bytes(c[0:4], "little") % 100 == 0:
            bit = int.from_bytes(c[4:6], "little") % 512
            sigc[i, bit // 8] ^= 1 << (bit % 8)
    assert hashlib.sha256(sigc.tobytes()).hexdigest() == g3["sha256_sig"]
    st3 = engine.ed25519_verify(msg, sigc, pk)
    assert hashlib.sha256(st3.tobytes()).hexdigest() == g3["sha256_status"]
    assert int((st3 == 0).sum()) == g3["accepted"]
