"""Host-side StatementBlock builder for benchmark corpora (configs 1, 4 and 5).

Mirrors block creation in the reference, `StatementBlock::new_with_signer`
(mysticeti-core/src/types.rs:155-218): the signer signs BLAKE2b-256 of the digest
pre-image (`Signer::sign_block`, crypto.rs:199-223), and the block digest is
BLAKE2b-256(pre-image || signature) (`BlockDigest::new`, crypto.rs:38-61). The bytes
are the `Data<StatementBlock>` bincode encoding (types.rs:93-114, data.rs:43-52).

Signing goes through the engine's batched GPU signer (`Engine.ed25519_sign`, the f3 row
of SURVEY.md §8): every authority of a round is signed in one call. The pre-image and
bincode writers here are independent of oracle/ (the checker); tests compare the two.
"""
from __future__ import annotations

import hashlib
import struct
from typing import List, Sequence, Tuple

import numpy as np

# (authority, round, digest) -- BlockReference (types.rs:49-54)
Ref = Tuple[int, int, bytes]


def _ref_bin(r: Ref) -> bytes:
    return struct.pack("<QQQ", r[0], r[1], 32) + r[2]


def _ref_pre(r: Ref) -> bytes:  # CryptoHash of BlockReference: BE authority, BE round, digest
    return struct.pack(">QQ", r[0], r[1]) + r[2]


def encode(author: int, rnd: int, includes: Sequence[Ref], shares: Sequence[bytes],
           ranges: Sequence[Tuple[Ref, int, int]], time_ns: int, epoch: int, sig: bytes,
           digest: bytes) -> Tuple[bytes, bytes]:
    """(bincode, pre-image) of a block whose statements are the Shares, then the VoteRanges.

    Pre-image: crypto.rs:85-128 (Share = 0x00 || raw tx, types.rs:751-755; VoteRange =
    0x04 || block || BE start || BE end; u128 BE time; marker byte; BE epoch).
    """
    pre = [struct.pack(">QQ", author, rnd)]
    bn = [struct.pack("<QQQ", author, rnd, 32), digest, struct.pack("<Q", len(includes))]
    for r in includes:
        pre.append(_ref_pre(r))
        bn.append(_ref_bin(r))
    bn.append(struct.pack("<Q", len(shares) + len(ranges)))
    for tx in shares:
        pre.append(b"\x00" + tx)
        bn.append(struct.pack("<IQ", 0, len(tx)) + tx)
    for r, lo, hi in ranges:
        pre.append(b"\x04" + _ref_pre(r) + struct.pack(">QQ", lo, hi))
        bn.append(struct.pack("<I", 2) + _ref_bin(r) + struct.pack("<QQ", lo, hi))
    pre.append(struct.pack(">QQ", time_ns >> 64, time_ns & (2**64 - 1)) + b"\x00" + struct.pack(">Q", epoch))
    bn.append(struct.pack("<QQ", time_ns & (2**64 - 1), time_ns >> 64) + b"\x00" + struct.pack("<QQ", epoch, 64))
    bn.append(sig)
    return b"".join(bn), b"".join(pre)


def _b2(x: bytes) -> bytes:
    return hashlib.blake2b(x, digest_size=32).digest()


def genesis_refs(n_auth: int, epoch: int = 0) -> List[Ref]:
    """References of the genesis blocks (types.rs:141-150): round 0, no includes, zero signature."""
    out = []
    for a in range(n_auth):
        _, pre = encode(a, 0, [], [], [], 0, epoch, bytes(64), bytes(32))
        out.append((a, 0, _b2(pre + bytes(64))))
    return out


def authority_seed(a: int) -> bytes:
    return hashlib.sha512(b"mysti-auth" + struct.pack("<Q", a)).digest()[:32]


def config4_tx(r: int, a: int) -> bytes:
    """512-B Share tx (transactions_generator.rs:82-85): 8-B ts || 8-B rand || zeros."""
    return (1_700_000_000_000 + r).to_bytes(8, "little") + \
        ((r * 1_000_003 + a * 7919) & (2**64 - 1)).to_bytes(8, "little") + bytes(496)


def build_rounds(engine, rounds: int, n_auth: int, seeds: Sequence[bytes], n_inc: int, n_vr: int,
                 with_tx: bool, epoch: int = 0) -> List[bytes]:
    """Rounds 1..rounds of a DAG: each authority includes n_inc blocks of round r-1 (own
    first, core.rs:264-278), optionally one 512-B Share tx, and n_vr VoteRanges. One GPU
    signing call per round."""
    prev = genesis_refs(n_auth, epoch)
    seed_arr = np.frombuffer(b"".join(seeds), dtype=np.uint8).reshape(n_auth, 32)
    out: List[bytes] = []
    for r in range(1, rounds + 1):
        specs, msgs = [], []
        for a in range(n_auth):
            others = [x for x in range(n_auth) if x != a]
            inc = [prev[a]] + [prev[x] for x in others[: n_inc - 1]]
            shares = [config4_tx(r, a)] if with_tx else []
            ranges = [(prev[(a + 1 + v) % n_auth], 0, 1 + (v % 7)) for v in range(n_vr)]
            t = r * 10**8 + a
            _, pre = encode(a, r, inc, shares, ranges, t, epoch, bytes(64), bytes(32))
            specs.append((a, inc, shares, ranges, t, pre))
            msgs.append(_b2(pre))
        _, sig = engine.ed25519_sign(seed_arr, np.frombuffer(b"".join(msgs), dtype=np.uint8).reshape(-1, 32))
        cur = []
        for (a, inc, shares, ranges, t, pre), s in zip(specs, sig):
            s = s.tobytes()
            d = _b2(pre + s)
            bn, _ = encode(a, r, inc, shares, ranges, t, epoch, s, d)
            out.append(bn)
            cur.append((a, r, d))
        prev = cur
    return out


def config1(engine, rounds: int) -> List[bytes]:
    """Config 1: 4 authorities, all with the zero seed (dummy_signer, crypto.rs:355-357)."""
    return build_rounds(engine, rounds, 4, [bytes(32)] * 4, n_inc=4, n_vr=0, with_tx=False)


def config4(engine, rounds: int, n_auth: int = 100, n_inc: int = 67, n_vr: int = 66) -> List[bytes]:
    """Config-4 shape: 100 authorities with distinct seeds, 67 includes, one 512-B tx and 66
    VoteRanges (pre-image ~8,060 B, bincode ~9.5 KB)."""
    return build_rounds(engine, rounds, n_auth, [authority_seed(a) for a in range(n_auth)], n_inc, n_vr,
                        with_tx=True)


def committee(engine, n_auth: int, distinct: bool):
    """(pks[n][32], stakes) of a corpus committee, public keys derived on the GPU."""
    seeds = [authority_seed(a) if distinct else bytes(32) for a in range(n_auth)]
    pk, _ = engine.ed25519_sign(np.frombuffer(b"".join(seeds), dtype=np.uint8).reshape(-1, 32),
                                np.zeros((n_auth, 32), dtype=np.uint8))
    return pk, np.ones(n_auth, dtype=np.uint64)


def pack(blocks: Sequence[bytes]):
    """(buf, off, len) arrays for Engine.verify_blocks_packed."""
    lens = np.array([len(b) for b in blocks], dtype=np.uint64)
    offs = np.zeros(len(blocks), dtype=np.uint64)
    if len(blocks) > 1:
        offs[1:] = np.cumsum(lens)[:-1]
    return np.frombuffer(b"".join(blocks) + b"\0", dtype=np.uint8), offs, lens
