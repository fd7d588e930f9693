"""The cofactored verdict of the comb kernels (comb.hip comb16_wg / k_comb_post) tests whether
R - S lies in the 8-torsion E[8] as X = 0 or Y = 0 or X^2 + Y^2 = 0 (quad25519.h
qp_in_torsion) instead of computing [8](R - S) and testing it for the identity, which is what
ed25519-consensus 2.1.0 does (mysticeti-core/src/crypto.rs:188, `verify` -> cofactored check).

This test pins the equivalence on affine edwards25519 arithmetic in Python integers: the
predicate holds on all eight points of E[8] and on none of a seeded sample of Q + T (Q a
nonzero multiple of the base point, T in E[8]), in projective scalings as well.
"""
import random

P = 2**255 - 19
D = (-121665 * pow(121666, P - 2, P)) % P
SQRTM1 = pow(2, (P - 1) // 4, P)
L = 2**252 + 27742317777372353535851937790883648493


def add(a, b):
    x1, y1 = a
    x2, y2 = b
    t = D * x1 * x2 * y1 * y2 % P
    return ((x1 * y2 + y1 * x2) * pow(1 + t, P - 2, P) % P, (y1 * y2 + x1 * x2) * pow(1 - t, P - 2, P) % P)


def mul(k, a):
    r = (0, 1)
    while k:
        if k & 1:
            r = add(r, a)
        a = add(a, a)
        k >>= 1
    return r


def decode_x(y, sign=0):
    x2 = (y * y - 1) * pow(D * y * y + 1, P - 2, P) % P
    x = pow(x2, (P + 3) // 8, P)
    if (x * x - x2) % P:
        x = x * SQRTM1 % P
    if (x * x - x2) % P:
        return None
    return P - x if (x & 1) != sign else x


def in_torsion(x, y, z=1):
    X, Y = x * z % P, y * z % P
    return X == 0 or Y == 0 or (X * X + Y * Y) % P == 0


def eight_torsion():
    rng = random.Random(7)
    while True:
        y = rng.randrange(P)
        x = decode_x(y)
        if x is None:
            continue
        t = mul(L, (x, y))  # kills the prime-order part
        pts = {mul(k, t) for k in range(8)}
        if len(pts) == 8:  # t generates E[8]
            return sorted(pts)


def test_predicate_matches_cofactored_identity_test():
    tors = eight_torsion()
    for t in tors:
        assert mul(8, t) == (0, 1)
        assert in_torsion(*t)
    by = 4 * pow(5, P - 2, P) % P
    base = (decode_x(by), by)
    rng = random.Random(11)
    for _ in range(40):
        q = mul(rng.randrange(1, L), base)
        for t in tors:
            p = add(q, t)
            assert mul(8, p) != (0, 1)
            z = rng.randrange(1, P)
            assert not in_torsion(p[0], p[1], z)
