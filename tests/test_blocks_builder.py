"""CPU: the product's bench-corpus block writer (mysticeti_amd/blocks.py) produces the same
bincode and digest pre-image as the oracle's model of Data<StatementBlock> (types.rs:93-114,
crypto.rs:85-128) and as the library's host codec."""
import hashlib

import numpy as np

import blocks as B
import mysticeti_amd.blocks as MB
import oracle as O


def test_encode_matches_oracle_model():
    rng = np.random.default_rng(9)
    for _ in range(20):
        a, r = int(rng.integers(0, 100)), int(rng.integers(1, 10**6))
        incs = [(int(rng.integers(0, 100)), r - 1, rng.integers(0, 256, 32, dtype=np.uint8).tobytes())
                for _ in range(int(rng.integers(0, 70)))]
        shares = [rng.integers(0, 256, int(rng.integers(0, 600)), dtype=np.uint8).tobytes()
                  for _ in range(int(rng.integers(0, 3)))]
        ranges = [(incs[0] if incs else (1, 2, bytes(32)), int(rng.integers(0, 5)), int(rng.integers(0, 9)))
                  for _ in range(int(rng.integers(0, 70)))]
        t = int(rng.integers(0, 2**62)) * (2**64 if rng.random() < 0.3 else 1)
        sig = rng.integers(0, 256, 64, dtype=np.uint8).tobytes()
        dig = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
        bn, pre = MB.encode(a, r, incs, shares, ranges, t, 0, sig, dig)
        ob = B.StatementBlock(a, r, [B.BlockReference(*x) for x in incs],
                              [("share", s) for s in shares] +
                              [("range", B.BlockReference(*x[0]), x[1], x[2]) for x in ranges],
                              t, False, 0, sig, dig)
        assert bn == ob.bincode()
        assert pre == ob.preimage() == O.block_preimage(bn)


def test_genesis_refs_match_oracle():
    for a, (ga, gr, gd) in enumerate(MB.genesis_refs(4)):
        g = B.genesis(a)
        assert (ga, gr, gd) == (g.authority, g.round, g.digest)


def test_config4_tx_layout():
    assert MB.config4_tx(3, 5) == B.config4_tx(3, 5)
    assert len(MB.config4_tx(1, 1)) == 512
    assert hashlib.sha256(MB.authority_seed(7)).digest() == hashlib.sha256(B.authority_seed(7)).digest()
