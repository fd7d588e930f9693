"""ORACLE / TEST INFRASTRUCTURE ONLY: Python model of Data<StatementBlock>.

Builds StatementBlocks byte-for-byte as the reference would serialize them and
computes their digests, for fixtures and parity tests:
  * bincode layout: types.rs:93-114 field order; BlockReference types.rs:49-54;
    BaseStatement types.rs:57-64; Vote types.rs:31-35; locators types.rs:384-394;
    SignatureBytes/BlockDigest as length-prefixed bytes (crypto.rs:309-347);
    bincode 1.3.3 defaults (LE, fixint, u64 lengths, u32 enum tags).
  * digest pre-image: crypto.rs:85-128 (+ CryptoHash impls crypto.rs:150-170,
    types.rs:661-691, types.rs:751-755).
  * block creation: StatementBlock::new_with_signer types.rs:155-218 (sign the
    Blake2b-256 of the pre-image, then digest = Blake2b-256(pre-image || sig));
    genesis types.rs:141-150 (round 0, no includes, zero signature).
  * corpora: config 1 (4 authorities, includes = the 4 blocks of round r-1, own
    first, core.rs:264-278) and the config-4 shape (100 authorities, 67 includes,
    one 512-B Share tx laid out as transactions_generator.rs:82-85, 66 VoteRanges).
Signing goes through a pluggable `signer(seed, msg32) -> sig64` so fixture
generation can use libsodium and tests can use the C oracle.
"""
from __future__ import annotations

import hashlib
import struct
from dataclasses import dataclass, field
from typing import Callable, List, Optional, Tuple


def b2b256(data: bytes) -> bytes:
    return hashlib.blake2b(data, digest_size=32).digest()


@dataclass(frozen=True)
class BlockReference:
    authority: int
    round: int
    digest: bytes

    def bincode(self) -> bytes:
        return struct.pack("<QQQ", self.authority, self.round, 32) + self.digest

    def preimage(self) -> bytes:
        return struct.pack(">QQ", self.authority, self.round) + self.digest


@dataclass(frozen=True)
class Locator:  # TransactionLocator
    block: BlockReference
    offset: int

    def bincode(self) -> bytes:
        return self.block.bincode() + struct.pack("<Q", self.offset)

    def preimage(self) -> bytes:
        return self.block.preimage() + struct.pack(">Q", self.offset)


# Statements: ("share", bytes) | ("accept", Locator) | ("reject", Locator, Optional[Locator])
#             | ("range", BlockReference, start, end)
Statement = tuple


def statement_bincode(st: Statement) -> bytes:
    kind = st[0]
    if kind == "share":
        return struct.pack("<IQ", 0, len(st[1])) + st[1]
    if kind == "accept":
        return struct.pack("<I", 1) + st[1].bincode() + struct.pack("<I", 0)
    if kind == "reject":
        out = struct.pack("<I", 1) + st[1].bincode() + struct.pack("<I", 1)
        if st[2] is None:
            return out + b"\x00"
        return out + b"\x01" + st[2].bincode()
    if kind == "range":
        return struct.pack("<I", 2) + st[1].bincode() + struct.pack("<QQ", st[2], st[3])
    raise ValueError(kind)


def statement_preimage(st: Statement) -> bytes:
    kind = st[0]
    if kind == "share":
        return b"\x00" + st[1]
    if kind == "accept":
        return b"\x01" + st[1].preimage()
    if kind == "reject":
        if st[2] is None:
            return b"\x02" + st[1].preimage()
        return b"\x03" + st[1].preimage() + st[2].preimage()
    if kind == "range":
        return b"\x04" + st[1].preimage() + struct.pack(">QQ", st[2], st[3])
    raise ValueError(kind)


@dataclass
class StatementBlock:
    authority: int
    round: int
    includes: List[BlockReference]
    statements: List[Statement]
    meta_creation_time_ns: int
    epoch_marker: bool
    epoch: int
    signature: bytes = bytes(64)
    digest: bytes = bytes(32)

    def preimage(self) -> bytes:
        out = [struct.pack(">QQ", self.authority, self.round)]
        out += [inc.preimage() for inc in self.includes]
        out += [statement_preimage(s) for s in self.statements]
        t = self.meta_creation_time_ns
        out.append(struct.pack(">QQ", t >> 64, t & (2**64 - 1)))
        out.append(b"\x01" if self.epoch_marker else b"\x00")
        out.append(struct.pack(">Q", self.epoch))
        return b"".join(out)

    def signed_message(self) -> bytes:
        return b2b256(self.preimage())

    def compute_digest(self) -> bytes:
        return b2b256(self.preimage() + self.signature)

    def reference(self) -> BlockReference:
        return BlockReference(self.authority, self.round, self.digest)

    def bincode(self) -> bytes:
        out = [struct.pack("<QQQ", self.authority, self.round, 32), self.digest]
        out.append(struct.pack("<Q", len(self.includes)))
        out += [inc.bincode() for inc in self.includes]
        out.append(struct.pack("<Q", len(self.statements)))
        out += [statement_bincode(s) for s in self.statements]
        t = self.meta_creation_time_ns
        out.append(struct.pack("<QQ", t & (2**64 - 1), t >> 64))
        out.append(b"\x01" if self.epoch_marker else b"\x00")
        out.append(struct.pack("<QQ", self.epoch, 64))
        out.append(self.signature)
        return b"".join(out)


Signer = Callable[[bytes, bytes], bytes]


def new_with_signer(authority, round_, includes, statements, time_ns, marker, epoch, seed: bytes,
                    signer: Signer) -> StatementBlock:
    b = StatementBlock(authority, round_, list(includes), list(statements), time_ns, marker, epoch)
    b.signature = signer(seed, b.signed_message())
    b.digest = b.compute_digest()
    return b


def genesis(authority: int, epoch: int = 0) -> StatementBlock:
    b = StatementBlock(authority, 0, [], [], 0, False, epoch)
    b.digest = b.compute_digest()
    return b


ZERO_SEED = bytes(32)  # dummy_signer(), crypto.rs:355-357


def authority_seed(a: int) -> bytes:
    return hashlib.sha512(b"mysti-auth" + struct.pack("<Q", a)).digest()[:32]


def gen_config1(signer: Signer, rounds: int = 1024, n_auth: int = 4) -> List[StatementBlock]:
    """Config 1: every authority signs with the zero seed, includes = the n_auth
    blocks of round r-1 with its own first, no statements, time = r*10^8 + a."""
    prev = [genesis(a) for a in range(n_auth)]
    out = []
    for r in range(1, rounds + 1):
        cur = []
        for a in range(n_auth):
            inc = [prev[a].reference()] + [prev[x].reference() for x in range(n_auth) if x != a]
            cur.append(new_with_signer(a, r, inc, [], r * 10**8 + a, False, 0, ZERO_SEED, signer))
        out += cur
        prev = cur
    return out


def config4_tx(r: int, a: int) -> bytes:
    """512-B Share tx laid out as transactions_generator.rs:82-85: 8-B ts || 8-B rand || zeros."""
    ts = (1_700_000_000_000 + r).to_bytes(8, "little")
    rnd = ((r * 1_000_003 + a * 7919) & (2**64 - 1)).to_bytes(8, "little")
    return ts + rnd + bytes(496)


def gen_config4(signer: Signer, rounds: int, n_auth: int = 100, n_inc: int = 67, n_vr: int = 66,
                first_round: int = 1) -> List[StatementBlock]:
    """Config-4 shape: distinct per-authority seeds, n_inc includes of round r-1
    (own first), one 512-B Share tx and n_vr VoteRange statements over the
    round r-1 blocks."""
    seeds = [authority_seed(a) for a in range(n_auth)]
    prev = [genesis(a) for a in range(n_auth)]
    out = []
    for r in range(first_round, first_round + rounds):
        cur = []
        for a in range(n_auth):
            others = [x for x in range(n_auth) if x != a]
            inc = [prev[a].reference()] + [prev[x].reference() for x in others[: n_inc - 1]]
            sts = [("share", config4_tx(r, a))]
            for v in range(n_vr):
                tgt = prev[(a + 1 + v) % n_auth].reference()
                sts.append(("range", tgt, 0, 1 + (v % 7)))
            cur.append(new_with_signer(a, r, inc, sts, r * 10**8 + a, False, 0, seeds[a], signer))
        out += cur
        prev = cur
    return out
