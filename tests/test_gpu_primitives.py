"""GPU: field / scalar / hash primitives of the HIP kernels vs Python big integers
and hashlib (bit-exact). Edge values: 0, 1, p-1, p, p+1, 2^255-1, 2^256-1, y+p."""
import hashlib
import random

import numpy as np
import pytest

import zip215 as Z

pytestmark = pytest.mark.gpu
P = Z.P
EDGE = [0, 1, 2, 19, P - 1, P, P + 1, P + 18, 2**255 - 1, 2**255, 2**256 - 1, 2**256 - 38, 2**32 - 1, 2**224,
        Z.D, Z.SQRT_M1]


def words(x: int, n=8):
    return [(x >> (32 * i)) & 0xFFFFFFFF for i in range(n)]


def val(ws):
    return sum(int(w) << (32 * i) for i, w in enumerate(ws))


def pairs(r, count=300):
    out = [(a, b) for a in EDGE for b in EDGE[:6]]
    for _ in range(count):
        out.append((r.randrange(2**256), r.randrange(2**256)))
    return out


def run(engine, op, items):
    w = np.array([words(a) + words(b) for a, b in items], dtype=np.uint32)
    return engine.selftest(op, w)


def test_fe_mul_sq_add_sub(engine):
    r = random.Random(1)
    items = pairs(r)
    for op, f in [(0, lambda a, b: a * b), (1, lambda a, b: a * a), (2, lambda a, b: a + b),
                  (6, lambda a, b: a * (b & 0x3FFFFFF))]:
        it = items if op != 6 else [(a, b & 0x3FFFFFF) for a, b in items]
        out = run(engine, op, it)
        for (a, b), o in zip(it, out):
            assert val(o[:8]) == f(a, b) % P, (op, a, b)


def test_fe_sub_tight_inputs(engine):
    # fe_sub's contract: tight inputs (< 2^255 + 2^14) -- which every fe op returns
    r = random.Random(2)
    items = [(a % (2**255 + 2**13), b % (2**255 + 2**13)) for a, b in pairs(r)]
    out = run(engine, 3, items)
    for (a, b), o in zip(items, out):
        assert val(o[:8]) == (a - b) % P, (a, b)


def test_fe_invert_pow(engine):
    r = random.Random(3)
    items = [(a, 0) for a in EDGE] + [(r.randrange(2**256), 0) for _ in range(100)]
    out = run(engine, 4, items)
    for (a, _), o in zip(items, out):
        assert val(o[:8]) == pow(a % P, P - 2, P)
    out = run(engine, 5, items)
    for (a, _), o in zip(items, out):
        assert val(o[:8]) == pow(a % P, (P - 5) // 8, P)


def test_fe_canon_of_255_bit_inputs(engine):
    items = [(y, 0) for y in [0, 1, P - 1, P, P + 1, P + 18, 2**255 - 1]]
    out = run(engine, 12, items)
    for (a, _), o in zip(items, out):
        assert val(o[:8]) == (a & (2**255 - 1)) % P


def test_decompress_zip215(engine):
    r = random.Random(4)
    encs = [e for e, _ in Z.small_order_encodings()]
    encs += [r.randrange(2**256).to_bytes(32, "little") for _ in range(200)]
    encs += [(y | s << 255).to_bytes(32, "little") for y in range(P, 2**255) for s in (0, 1)]
    w = np.array([list(np.frombuffer(e, dtype=np.uint32)) + [0] * 8 for e in encs], dtype=np.uint32)
    out = engine.selftest(7, w)
    for e, o in zip(encs, out):
        pt = Z.decompress(e)
        assert bool(o[8]) == (pt is not None), e.hex()
        if pt is not None:
            assert val(o[:8]) == pt[0] % P, e.hex()


def test_scalar_reduce_and_canonical(engine):
    r = random.Random(5)
    xs = [0, 1, Z.L - 1, Z.L, Z.L + 1, 2 * Z.L, 2**512 - 1, 2**256, Z.L * Z.L] + [r.randrange(2**512) for _ in range(300)]
    w = np.array([words(x, 16) for x in xs], dtype=np.uint32)
    out = engine.selftest(8, w)
    for x, o in zip(xs, out):
        assert val(o[:8]) == x % Z.L
    ss = [0, 1, Z.L - 1, Z.L, Z.L + 1, 2**255 - 1, 2**253, 2**252] + [r.randrange(2**256) for _ in range(100)]
    w = np.array([words(s) + [0] * 8 for s in ss], dtype=np.uint32)
    out = engine.selftest(10, w)
    for s, o in zip(ss, out):
        assert o[0] == (1 if s < Z.L else 0), s


def test_sha512_64(engine):
    r = random.Random(6)
    msgs = [bytes(r.randrange(256) for _ in range(64)) for _ in range(100)]
    w = np.array([list(np.frombuffer(m, dtype=np.uint32)) for m in msgs], dtype=np.uint32)
    out = engine.selftest(9, w)
    for m, o in zip(msgs, out):
        assert o.astype("<u4").tobytes() == hashlib.sha512(m).digest()


def test_quad_lane_field_ops(engine):
    """fe_q4.h (four lanes per element, the online path's R decode): products, the
    (p-5)/8 power and 50 repeated squarings, against Python big integers, on edge values and
    random ones. Every lane of a quad carries the same input."""
    r = random.Random(8)
    items = pairs(r, 200)
    rep = [it for it in items for _ in range(4)]
    out = run(engine, 16, rep)
    for k, (a, b) in enumerate(items):
        want = (a % 2**256) * (b % 2**256) % P
        for j in range(4):
            assert val(out[4 * k + j][:8]) == want, (a, b, j)
    out = run(engine, 17, rep)
    for k, (a, b) in enumerate(items):
        want = pow(a % 2**256, (P - 5) // 8, P)
        assert val(out[4 * k][:8]) == want, a
        assert all(val(out[4 * k + j][:8]) == want for j in range(4))
    out = run(engine, 18, rep)
    for k, (a, b) in enumerate(items):
        assert val(out[4 * k][:8]) == pow(a % 2**256, 2**50, P), a


def test_row_lane_field_ops(engine):
    """fe_r16.h (one 16-lane DPP row per element, the online path's R decode): products, the
    (p-5)/8 power and 50 repeated squarings, against Python big integers, on edge values and
    random ones. Every lane of a row carries the same input (whole rows: 16 copies)."""
    r = random.Random(9)
    items = pairs(r, 200)
    rep = [it for it in items for _ in range(16)]
    out = run(engine, 19, rep)
    for k, (a, b) in enumerate(items):
        want = (a % 2**256) * (b % 2**256) % P
        for j in range(16):
            assert val(out[16 * k + j][:8]) == want, (a, b, j)
    out = run(engine, 20, rep)
    for k, (a, b) in enumerate(items):
        want = pow(a % 2**256, (P - 5) // 8, P)
        assert all(val(out[16 * k + j][:8]) == want for j in range(16)), a
    out = run(engine, 21, rep)
    for k, (a, b) in enumerate(items):
        assert val(out[16 * k][:8]) == pow(a % 2**256, 2**50, P), a


def test_sha512_96(engine):
    """The 96-byte form the challenge k = SHA-512(R || A || M) uses (crypto.rs:188 via
    ed25519-consensus): selftest op 15 hashes the 64 input bytes followed by their first 32."""
    r = random.Random(7)
    msgs = [bytes(r.randrange(256) for _ in range(64)) for _ in range(100)]
    msgs += [bytes(64), bytes([0xff]) * 64]
    w = np.array([list(np.frombuffer(m, dtype=np.uint32)) for m in msgs], dtype=np.uint32)
    out = engine.selftest(15, w)
    for m, o in zip(msgs, out):
        assert o.astype("<u4").tobytes() == hashlib.sha512(m + m[:32]).digest()


def test_basepoint_mul(engine):
    r = random.Random(8)
    ks = [0, 1, 2, 3, 127, 128, 129, 255, 256, Z.L - 1] + [r.randrange(Z.L) for _ in range(60)]
    w = np.array([words(k) + [0] * 8 for k in ks], dtype=np.uint32)
    out = engine.selftest(11, w)
    for k, o in zip(ks, out):
        assert o[:8].astype("<u4").tobytes() == Z.compress(Z.scalarmult(Z.B_POINT, k)), k


def test_blake2b_kats(engine, golden):
    g = golden("hash_kat.json")
    lens = [int(n) for n in g["blake2b256"]]
    items = [bytes((i * 31 + 7) % 251 for i in range(n)) for n in lens]
    out = engine.blake2b256(items)
    for n, o in zip(lens, out):
        assert o.hex() == g["blake2b256"][str(n)], n


def _halfsize_model(k):
    """Extended-Euclid remainder sequence of (l, k) stopped below 2^126, quotients as
    shift-subtract steps (the algorithm of scalar25519.h sc_halfsize)."""
    a, ta, b, tb = Z.L, 0, k, 1
    if b < 2**126:
        return b, 1
    while True:
        s = a.bit_length() - b.bit_length()
        if (b << s) > a:
            s -= 1
        a -= b << s
        ta -= tb << s
        if a < 2**126:
            return a, ta
        if a < b:
            a, ta, b, tb = b, tb, a, ta


def test_halfsize_scalars(engine):
    r = random.Random(9)
    T = 2**126
    ks = [0, 1, 2, T - 1, T, T + 1, 2**200 + 5, 2**252, Z.L - 1, Z.L - 2, (Z.L - 1) // 2, (Z.L + 1) // 2,
          2**252 - 1, 3 * T, Z.L // 3, Z.L // 5 + 7] + [r.randrange(Z.L) for _ in range(3000)]
    w = np.array([words(k) + [0] * 8 for k in ks], dtype=np.uint32)
    out = engine.selftest(13, w)
    for k, o in zip(ks, out):
        c, neg, d = val(o[:4]), int(o[4]), val(o[8:12])
        mc, md = _halfsize_model(k)
        if md < 0:
            mc, md = -mc, -md
        assert (-c if neg else c) == mc and d == md, k
        # the property the verify equation relies on
        assert ((-c if neg else c) - d * k) % Z.L == 0 and c < T and 0 < d < 2**127, k
        assert (d >> 124) <= 6  # the radix-16 recoding's top digit stays in [-8, 7]


def test_second_fixed_base_table(engine):
    # [a](2^124 B) from the second LDS table == [a * 2^124 mod l]B
    r = random.Random(10)
    ks = [0, 1, 2, 128, 129, Z.L - 1] + [r.randrange(Z.L) for _ in range(60)]
    w = np.array([words(k) + [0] * 8 for k in ks], dtype=np.uint32)
    out = engine.selftest(14, w)
    for k, o in zip(ks, out):
        assert o[:8].astype("<u4").tobytes() == Z.compress(Z.scalarmult(Z.B_POINT, k * 2**124 % Z.L)), k


def test_blake2b_ragged_lengths(engine):
    """Every length 0..700 and some up to 40 KB in one call: the 16 strings of a quad-kernel
    workgroup run different step counts (RFC 7693, checked with hashlib)."""
    import hashlib

    rng = np.random.default_rng(9)
    lens = list(range(0, 701)) + [int(x) for x in rng.integers(700, 40000, size=60)]
    rng.shuffle(lens)
    items = [rng.integers(0, 256, size=n, dtype=np.uint8).tobytes() for n in lens]
    out = engine.blake2b256(items)
    for it, o in zip(items, out):
        assert bytes(o) == hashlib.blake2b(it, digest_size=32).digest(), len(it)


def test_blake2b_ragged_lengths_batch_size(engine):
    """A batch-size call (>= MV_BATCH_MIN strings: the lane-per-string kernel, blake2b_lane.hip)
    with ragged lengths, empty and block-boundary strings among them (checked with hashlib)."""
    import hashlib

    rng = np.random.default_rng(11)
    lens = [0, 1, 127, 128, 129, 255, 256, 257, 8060, 8124] + [int(x) for x in rng.integers(0, 3000, size=4200)]
    rng.shuffle(lens)
    items = [rng.integers(0, 256, size=n, dtype=np.uint8).tobytes() for n in lens]
    out = engine.blake2b256(items)
    for it, o in zip(items, out):
        assert bytes(o) == hashlib.blake2b(it, digest_size=32).digest(), len(it)
