"""ORACLE / TEST INFRASTRUCTURE ONLY — never imported by the product path.

Pure-Python big-integer restatement of the signature path the reference calls:

* ``ed25519-consensus 2.1.0`` (``Cargo.lock:917``), called at
  ``mysticeti-core/src/crypto.rs:188`` (``VerificationKey::verify``) and
  ``crypto.rs:221`` (``SigningKey::sign``). The crate is not vendored under
  /root/reference; its published algorithm is restated here:
    - ZIP-215 decoding: y is read from 255 bits WITHOUT a range check (y >= p is
      reduced mod p), x is recovered by the dalek ``sqrt_ratio_i`` rule, the sign
      bit negates x even when x == 0.
    - ``s`` must be canonical (< l, ``Scalar::from_canonical_bytes``).
    - k = SHA-512(R_bytes || A_bytes || msg) mod l over the ORIGINAL bytes.
    - accept  <=>  [8](R - ([s]B - [k]A)) == identity  (cofactored).
* ``curve25519-dalek-ng 4.1.1`` (``Cargo.lock:842``) field / point semantics.
* RFC 8032 deterministic signing (used only to build corpora; cross-checked
  against libsodium in ``oracle/gen_fixtures.py``).

Small cases only (a verify costs ~5 ms here). The fast CPU restatement is the C
oracle in ``oracle/ed25519_oracle.c``; both are pinned by ``tests/golden``.
"""
from __future__ import annotations

import hashlib

P = 2**255 - 19
L = 2**252 + 27742317777372353535851937790883648493
D = (-121665 * pow(121666, P - 2, P)) % P
D2 = (2 * D) % P
SQRT_M1 = pow(2, (P - 1) // 4, P)


def _inv(x: int) -> int:
    return pow(x, P - 2, P)


def is_negative(x: int) -> bool:
    """dalek ``FieldElement::is_negative``: low bit of the canonical encoding."""
    return (x % P) & 1 == 1


def sqrt_ratio_i(u: int, v: int):
    """dalek ``FieldElement::sqrt_ratio_i`` (returns (was_nonzero_square_or_zero, r>=0))."""
    u %= P
    v %= P
    v3 = v * v % P * v % P
    v7 = v3 * v3 % P * v % P
    r = u * v3 % P * pow(u * v7 % P, (P - 5) // 8, P) % P
    check = v * r % P * r % P
    correct = check == u
    flipped = check == (-u) % P
    flipped_i = check == (-u) * SQRT_M1 % P
    if flipped or flipped_i:
        r = r * SQRT_M1 % P
    if is_negative(r):
        r = (-r) % P
    return (correct or flipped), r


# Points are extended twisted-Edwards tuples (X, Y, Z, T), x = X/Z, y = Y/Z, xy = T/Z.
IDENTITY = (0, 1, 1, 0)


def decompress(b: bytes):
    """ZIP-215 / dalek ``CompressedEdwardsY::decompress``; None if not on the curve."""
    assert len(b) == 32
    y = int.from_bytes(b, "little") & ((1 << 255) - 1)
    sign = b[31] >> 7
    y %= P  # non-canonical y (>= p) accepted, reduced
    yy = y * y % P
    u = (yy - 1) % P
    v = (D * yy + 1) % P
    ok, x = sqrt_ratio_i(u, v)
    if not ok:
        return None
    if sign:
        x = (-x) % P  # x == 0 with the sign bit set is accepted
    return (x, y, 1, x * y % P)


def compress(pt) -> bytes:
    X, Y, Z, _ = pt
    zi = _inv(Z)
    x = X * zi % P
    y = Y * zi % P
    return (y | ((x & 1) << 255)).to_bytes(32, "little")


def add(p1, p2):
    """Unified addition for a = -1 (add-2008-hwcd-3)."""
    X1, Y1, Z1, T1 = p1
    X2, Y2, Z2, T2 = p2
    A = (Y1 - X1) * (Y2 - X2) % P
    B = (Y1 + X1) * (Y2 + X2) % P
    C = T1 * D2 % P * T2 % P
    Dd = 2 * Z1 * Z2 % P
    E, F, G, H = B - A, Dd - C, Dd + C, B + A
    return (E * F % P, G * H % P, F * G % P, E * H % P)


def neg(pt):
    X, Y, Z, T = pt
    return ((-X) % P, Y, Z, (-T) % P)


def double(pt):
    return add(pt, pt)


def scalarmult(pt, k: int):
    q = IDENTITY
    for bit in bin(k)[2:] if k > 0 else "":
        q = double(q)
        if bit == "1":
            q = add(q, pt)
    return q


def is_identity(pt) -> bool:
    X, Y, Z, _ = pt
    return X % P == 0 and (Y - Z) % P == 0


def point_eq(p1, p2) -> bool:
    X1, Y1, Z1, _ = p1
    X2, Y2, Z2, _ = p2
    return (X1 * Z2 - X2 * Z1) % P == 0 and (Y1 * Z2 - Y2 * Z1) % P == 0


_By = 4 * _inv(5) % P
B_POINT = decompress(_By.to_bytes(32, "little"))
assert B_POINT is not None and not is_negative(B_POINT[0])


def sha512_mod_l(*parts: bytes) -> int:
    h = hashlib.sha512()
    for p in parts:
        h.update(p)
    return int.from_bytes(h.digest(), "little") % L


# ---- verification status codes (mirror include/mysti_verify.h MV_SIG_*) ----
SIG_OK = 0
SIG_INVALID = 1          # ed25519_consensus::Error::InvalidSignature
SIG_MALFORMED_KEY = 2    # ed25519_consensus::Error::MalformedPublicKey


def verify_status(pk: bytes, sig: bytes, msg: bytes) -> int:
    """ed25519-consensus 2.1.0 ``VerificationKey::try_from`` + ``verify`` (ZIP-215)."""
    A = decompress(pk)
    if A is None:
        return SIG_MALFORMED_KEY
    s = int.from_bytes(sig[32:], "little")
    if s >= L:  # also covers the high bit (s >= 2^255 > l)
        return SIG_INVALID
    R = decompress(sig[:32])
    if R is None:
        return SIG_INVALID
    k = sha512_mod_l(sig[:32], pk, msg)
    r_prime = add(scalarmult(B_POINT, s), neg(scalarmult(A, k)))
    diff = add(R, neg(r_prime))
    for _ in range(3):
        diff = double(diff)
    return SIG_OK if is_identity(diff) else SIG_INVALID


def verify(pk: bytes, sig: bytes, msg: bytes) -> bool:
    return verify_status(pk, sig, msg) == SIG_OK


def _clamp(h: bytes) -> int:
    a = bytearray(h[:32])
    a[0] &= 248
    a[31] &= 127
    a[31] |= 64
    return int.from_bytes(a, "little")


def public_key(seed: bytes) -> bytes:
    h = hashlib.sha512(seed).digest()
    return compress(scalarmult(B_POINT, _clamp(h)))


def sign(seed: bytes, msg: bytes) -> bytes:
    """RFC 8032 Ed25519 signing (== ed25519_consensus::SigningKey::sign)."""
    h = hashlib.sha512(seed).digest()
    a = _clamp(h)
    A = compress(scalarmult(B_POINT, a))
    r = sha512_mod_l(h[32:], msg)
    R = compress(scalarmult(B_POINT, r))
    k = sha512_mod_l(R, A, msg)
    S = (r + k * a) % L
    return R + S.to_bytes(32, "little")


# ---- the eight torsion points and their encodings (ZIP-215 edge corpus) ----

def torsion_points():
    """All 8 points of E[8], found as (l * random point) multiples."""
    # A point of order 8: x^2 = (y^2-1)/(d y^2+1) with y chosen so order is 8.
    pts = {}
    seed = 0
    while len(pts) < 8:
        seed += 1
        y = int.from_bytes(hashlib.sha256(b"tors" + bytes([seed])).digest(), "little") % P
        cand = decompress(y.to_bytes(32, "little"))
        if cand is None:
            continue
        t = scalarmult(cand, L)
        q = t
        for _ in range(8):
            enc = compress(q)
            pts[enc] = q
            q = add(q, t)
    return pts


def small_order_encodings():
    """Canonical + non-canonical 32-byte encodings of every small-order point.

    Non-canonical forms: y + p for y < 19 (fits in 255 bits) and the sign bit set
    on x == 0 points. Each entry: (encoding bytes, canonical: bool).
    """
    out = []
    for enc, pt in sorted(torsion_points().items()):
        out.append((enc, True))
        x = pt[0] * _inv(pt[2]) % P
        y = pt[1] * _inv(pt[2]) % P
        if y + P < 2**255:
            ync = y + P
            out.append(((ync | ((x & 1) << 255)).to_bytes(32, "little"), False))
        if x == 0:
            out.append(((y | (1 << 255)).to_bytes(32, "little"), False))
            if y + P < 2**255:
                out.append((((y + P) | (1 << 255)).to_bytes(32, "little"), False))
    return out
