"""ORACLE / TEST INFRASTRUCTURE ONLY: generates tests/golden/* in the survey container.

Independent sources (none of them our C oracle or the product):
  * hashlib.blake2b(digest_size=32) / hashlib.sha512 (CPython's reference C code);
  * libsodium 1.0.18 (/opt/conda/lib/libsodium.so.23, ctypes): RFC 8032 deterministic
    signing == ed25519_consensus::SigningKey::sign; its strict verify is used only
    for ordinary (non-edge) signatures, where strict and ZIP-215 agree;
  * oracle/zip215.py: pure-Python big-integer ZIP-215 predicate for edge cases.
The reference's own tests hold no crypto vectors (crypto.rs:63-75,191-194,225-237
stub crypto under cfg(test)), so these fixtures are the parity anchor.

Usage: python oracle/gen_fixtures.py [--skip-1m]
"""
from __future__ import annotations

import argparse
import ctypes
import hashlib
import json
import multiprocessing as mp
import os
import struct
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import blocks as B  # noqa: E402
import zip215 as Z  # noqa: E402

GOLDEN = os.path.join(os.path.dirname(HERE), "tests", "golden")
SODIUM = "/opt/conda/lib/libsodium.so.23"
_sodium = None


def sodium():
    global _sodium
    if _sodium is None:
        _sodium = ctypes.CDLL(SODIUM)
        assert _sodium.sodium_init() >= 0
    return _sodium


def sodium_keypair(seed: bytes):
    pk = ctypes.create_string_buffer(32)
    sk = ctypes.create_string_buffer(64)
    sodium().crypto_sign_seed_keypair(pk, sk, seed)
    return pk.raw, sk.raw


def sodium_sign(seed: bytes, msg: bytes) -> bytes:
    _, sk = sodium_keypair(seed)
    sig = ctypes.create_string_buffer(64)
    n = ctypes.c_ulonglong()
    sodium().crypto_sign_detached(sig, ctypes.byref(n), msg, ctypes.c_ulonglong(len(msg)), sk)
    return sig.raw


def sodium_verify(pk: bytes, sig: bytes, msg: bytes) -> bool:
    return sodium().crypto_sign_verify_detached(sig, msg, ctypes.c_ulonglong(len(msg)), pk) == 0


def kat_input(n: int) -> bytes:
    return bytes((i * 31 + 7) % 251 for i in range(n))


def sha256hex(b: bytes) -> str:
    return hashlib.sha256(b).hexdigest()


# ---------------------------------------------------------------- hashes
def gen_hash_kat():
    lens = list(range(0, 260)) + [383, 384, 385, 511, 512, 513, 1000, 4096, 8060, 8124, 9999]
    g0 = B.genesis(0)
    return {
        "input": "bytes((i * 31 + 7) % 251 for i in range(len))",
        "blake2b256": {str(n): hashlib.blake2b(kat_input(n), digest_size=32).hexdigest() for n in lens},
        "sha512": {str(n): hashlib.sha512(kat_input(n)).hexdigest() for n in lens},
        "genesis_A0": {"preimage_hex": g0.preimage().hex(), "msg": g0.signed_message().hex(),
                       "digest": g0.digest.hex()},
        "genesis_B0_digest": B.genesis(1).digest.hex(),
        "zero_seed_pk": sodium_keypair(bytes(32))[0].hex(),
    }


# ---------------------------------------------------------------- signatures
def gen_sig_kat():
    out = []
    for i in range(64):
        seed = hashlib.sha512(b"kat-seed" + struct.pack("<Q", i)).digest()[:32]
        msg = hashlib.blake2b(b"kat-msg" + struct.pack("<Q", i), digest_size=32).digest()
        pk, _ = sodium_keypair(seed)
        sig = sodium_sign(seed, msg)
        assert Z.sign(seed, msg) == sig and Z.public_key(seed) == pk
        assert sodium_verify(pk, sig, msg) and Z.verify(pk, sig, msg)
        out.append({"seed": seed.hex(), "msg": msg.hex(), "pk": pk.hex(), "sig": sig.hex()})
    return out


def gen_zip215_corpus():
    """Edge cases with their ZIP-215 verdicts (status: 0 ok, 1 invalid sig, 2 malformed key)."""
    cases = []

    def add(pk, sig, msg, note):
        st = Z.verify_status(pk, sig, msg)
        cases.append({"pk": pk.hex(), "sig": sig.hex(), "msg": msg.hex(), "status": st, "note": note})

    enc = Z.small_order_encodings()
    # 1. every (A, R) pair of small-order encodings with s = 0: all accepted (ZIP-215).
    for a, ca in enc:
        for r, cr in enc:
            add(a, r + bytes(32), b"Zcash", f"small-order A{'c' if ca else 'nc'} R{'c' if cr else 'nc'} s=0")
    seed = hashlib.sha512(b"edge-seed").digest()[:32]
    pk, _ = sodium_keypair(seed)
    msg = hashlib.blake2b(b"edge-msg", digest_size=32).digest()
    sig = sodium_sign(seed, msg)
    add(pk, sig, msg, "valid")
    s = int.from_bytes(sig[32:], "little")
    # 2. non-canonical / out-of-range s
    for name, sv in [("s=l", Z.L), ("s=l+1", Z.L + 1), ("s+l", s + Z.L), ("s=2^255-1", 2**255 - 1),
                     ("s=2^253", 2**253), ("s=l-1", Z.L - 1), ("s=0", 0)]:
        add(pk, sig[:32] + sv.to_bytes(32, "little"), msg, name)
    add(pk, sig[:32] + (s | (1 << 255)).to_bytes(32, "little"), msg, "s high bit set")
    # 3. undecodable R / A (first y values whose (y^2-1)/(dy^2+1) is a non-square)
    bad = []
    y = 2
    while len(bad) < 4:
        e = y.to_bytes(32, "little")
        if Z.decompress(e) is None:
            bad.append(e)
        y += 1
    for e in bad:
        add(pk, e + sig[32:], msg, "R undecodable")
        add(e, sig, msg, "A undecodable (MalformedPublicKey)")
    # non-canonical y >= p that does not decode
    for yy in range(Z.P, 2**255):
        e = yy.to_bytes(32, "little")
        if Z.decompress(e) is None:
            add(pk, e + sig[32:], msg, "R y>=p undecodable")
            add(e, sig, msg, "A y>=p undecodable")
            break
    # 4. mixed-order R: R = rB + T (T of order 8), S re-derived: cofactored accept.
    tors = [p for enc_, p in Z.torsion_points().items() if not Z.is_identity(p)]
    h = hashlib.sha512(seed).digest()
    a_sc = Z._clamp(h)
    A = Z.scalarmult(Z.B_POINT, a_sc)
    assert Z.compress(A) == pk
    for ti, T in enumerate(tors[:4]):
        r = Z.sha512_mod_l(b"mixed", bytes([ti]))
        Rm = Z.add(Z.scalarmult(Z.B_POINT, r), T)
        Rb = Z.compress(Rm)
        k = Z.sha512_mod_l(Rb, pk, msg)
        S = (r + k * a_sc) % Z.L
        add(pk, Rb + S.to_bytes(32, "little"), msg, f"mixed-order R (torsion {ti})")
    # 5. mixed-order A: A' = A + T, signature with a: [8](SB - kA' - R) = [8](-kT) = 0.
    for ti, T in enumerate(tors[:4]):
        Ap = Z.compress(Z.add(A, T))
        r = Z.sha512_mod_l(b"mixedA", bytes([ti]))
        Rb = Z.compress(Z.scalarmult(Z.B_POINT, r))
        k = Z.sha512_mod_l(Rb, Ap, msg)
        S = (r + k * a_sc) % Z.L
        add(Ap, Rb + S.to_bytes(32, "little"), msg, f"mixed-order A (torsion {ti})")
    # 6. small-order A with a real R and s: accepted iff [8](sB - R) == 0 -> reject
    add(enc[0][0], sig, msg, "small-order A, real signature")
    # 7. non-canonical A encoding of a real key (x sign flipped -> a different point)
    add(pk[:31] + bytes([pk[31] ^ 0x80]), sig, msg, "A sign bit flipped")
    # 8. single-bit corruptions of R, s and the message
    for bit in [0, 7, 100, 254, 255, 256, 300, 383, 500, 511]:
        b = bytearray(sig)
        b[bit // 8] ^= 1 << (bit % 8)
        add(pk, bytes(b), msg, f"sig bit {bit} flipped")
    for bit in [0, 128, 255]:
        m = bytearray(msg)
        m[bit // 8] ^= 1 << (bit % 8)
        add(pk, sig, bytes(m), f"msg bit {bit} flipped")
    # 9. identity R with s = 0 for a real key: [8](0 - 0 - kA) = 0 only if kA small: reject
    add(pk, enc[0][0] + bytes(32), msg, "R=identity s=0 real key")
    return cases


# ---------------------------------------------------------------- 1M batch (configs 2 and 3)
def corpus_seed(i: int) -> bytes:
    return hashlib.sha512(b"mysti-seed" + struct.pack("<Q", i)).digest()[:32]


def corpus_msg(i: int) -> bytes:
    return hashlib.blake2b(b"mysti-msg" + struct.pack("<Q", i), digest_size=32).digest()


def corrupt_bit(i: int):
    """Config 3: 1% of signatures get one bit of R||s flipped (None if untouched)."""
    c = hashlib.sha256(b"mysti-corrupt" + struct.pack("<Q", i)).digest()
    if int.from_bytes(c[0:4], "little") % 100 != 0:
        return None
    return int.from_bytes(c[4:6], "little") % 512


def _sign_range(args):
    lo, hi = args
    pks, sigs = bytearray(), bytearray()
    for i in range(lo, hi):
        seed = corpus_seed(i)
        pk, _ = sodium_keypair(seed)
        pks += pk
        sigs += sodium_sign(seed, corpus_msg(i))
    return bytes(pks), bytes(sigs)


def _sodium_verify_range(args):
    pk, sig, msg = args
    n = len(pk) // 32
    return bytes(0 if sodium_verify(pk[32 * i:32 * i + 32], sig[64 * i:64 * i + 64], msg[32 * i:32 * i + 32])
                 else 1 for i in range(n))


def gen_batch(n: int):
    chunks = [(i, min(n, i + 16384)) for i in range(0, n, 16384)]
    with mp.Pool(8) as pool:
        res = pool.map(_sign_range, chunks)
    pk = b"".join(r[0] for r in res)
    sig = b"".join(r[1] for r in res)
    msg = b"".join(corpus_msg(i) for i in range(n))
    # pin: every signature verifies under libsodium (ordinary signatures: strict == ZIP-215)
    vchunks = [(pk[32 * lo:32 * hi], sig[64 * lo:64 * hi], msg[32 * lo:32 * hi]) for lo, hi in chunks]
    with mp.Pool(8) as pool:
        st = b"".join(pool.map(_sodium_verify_range, vchunks))
    assert st == bytes(n), "libsodium rejected a generated signature"
    spec = {
        "n": n,
        "seed_i": "SHA-512(b'mysti-seed' || u64le(i))[:32]",
        "msg_i": "Blake2b-256(b'mysti-msg' || u64le(i))",
        "sig_i": "RFC 8032 sign(seed_i, msg_i) (libsodium crypto_sign_detached)",
        "sha256_pk": sha256hex(pk), "sha256_sig": sha256hex(sig), "sha256_msg": sha256hex(msg),
        "sha256_status": sha256hex(st), "accepted": n,
    }
    # config 3: corruptions; verdicts from the pure-Python ZIP-215 predicate
    sig_c = bytearray(sig)
    status_c = bytearray(n)
    corrupted = []
    for i in range(n):
        bit = corrupt_bit(i)
        if bit is None:
            continue
        sig_c[64 * i + bit // 8] ^= 1 << (bit % 8)
        corrupted.append(i)
    for i in corrupted:
        status_c[i] = Z.verify_status(pk[32 * i:32 * i + 32], bytes(sig_c[64 * i:64 * i + 64]),
                                      msg[32 * i:32 * i + 32])
    spec_c = {
        "n": n, "corruption": "c = SHA-256(b'mysti-corrupt' || u64le(i)); corrupted iff u32le(c[0:4]) % 100 == 0; "
                              "bit = u16le(c[4:6]) % 512 of R||s flipped",
        "n_corrupted": len(corrupted), "sha256_sig": sha256hex(bytes(sig_c)), "sha256_status": sha256hex(bytes(status_c)),
        "accepted": int(n - sum(1 for s in status_c if s != 0)),
        "first_corrupted": {str(i): int(status_c[i]) for i in corrupted[:64]},
    }
    return spec, spec_c


# ---------------------------------------------------------------- blocks
def committee_zero(n):
    return {"pks": [sodium_keypair(B.ZERO_SEED)[0].hex()] * n, "stakes": [1] * n, "epoch": 0}


def gen_blocks_config1():
    blks = B.gen_config1(sodium_sign)
    bins = [b.bincode() for b in blks]
    msgs = b"".join(b.signed_message() for b in blks)
    digs = b"".join(b.digest for b in blks)
    pk = sodium_keypair(B.ZERO_SEED)[0]
    for b in blks[:64]:
        assert sodium_verify(pk, b.signature, b.signed_message())
    return {
        "committee": committee_zero(4),
        "n": len(blks),
        "sha256_bincode_concat": sha256hex(b"".join(bins)),
        "sha256_msg_digests": sha256hex(msgs),
        "sha256_block_digests": sha256hex(digs),
        "bincode_len_total": sum(len(x) for x in bins),
        "statuses": "all 0 (OK)",
        "first": [{"bincode": bins[i].hex(), "preimage": blks[i].preimage().hex(), "msg": blks[i].signed_message().hex(),
                   "digest": blks[i].digest.hex()} for i in range(8)],
    }


def gen_blocks_config4_sample():
    blks = B.gen_config4(sodium_sign, rounds=2)
    bins = [b.bincode() for b in blks]
    return {
        "committee": {"pks": [sodium_keypair(B.authority_seed(a))[0].hex() for a in range(100)],
                      "stakes": [1] * 100, "epoch": 0},
        "rounds": 2, "n": len(blks),
        "sha256_bincode_concat": sha256hex(b"".join(bins)),
        "sha256_msg_digests": sha256hex(b"".join(b.signed_message() for b in blks)),
        "sha256_block_digests": sha256hex(b"".join(b.digest for b in blks)),
        "bincode_len_first": len(bins[0]), "preimage_len_first": len(blks[0].preimage()),
        "first_msg": blks[0].signed_message().hex(), "first_digest": blks[0].digest.hex(),
    }


def gen_block_edge():
    """Mutated config-1 blocks with the status StatementBlock::verify (types.rs:315-376) returns."""
    blks = B.gen_config1(sodium_sign, rounds=3)
    base = blks[4]  # round 2, authority 0
    cases = []

    def add(b_bytes: bytes, status: int, note: str):
        cases.append({"bincode": b_bytes.hex(), "status": status, "note": note})

    def resign(b):
        b.signature = sodium_sign(B.ZERO_SEED, b.signed_message())
        b.digest = b.compute_digest()
        return b

    import copy
    add(base.bincode(), 0, "valid")
    b = copy.deepcopy(base); b.digest = bytes([b.digest[0] ^ 1]) + b.digest[1:]
    add(b.bincode(), 2, "digest mismatch")
    b = copy.deepcopy(base); b.epoch = 1; resign(b)
    add(b.bincode(), 3, "epoch mismatch")
    b = copy.deepcopy(base); b.authority = 4; resign(b)
    add(b.bincode(), 4, "unknown author")
    b = copy.deepcopy(base); b.round = 0; b.includes = []; resign(b)
    add(b.bincode(), 5, "genesis round")
    b = copy.deepcopy(base); b.signature = bytes([b.signature[0] ^ 4]) + b.signature[1:]; b.digest = b.compute_digest()
    add(b.bincode(), 6, "bad signature (digest recomputed)")
    b = copy.deepcopy(base); b.signature = b.signature[:32] + Z.L.to_bytes(32, "little"); b.digest = b.compute_digest()
    add(b.bincode(), 6, "s = l")
    b = copy.deepcopy(base); b.includes = b.includes + [B.BlockReference(9, 1, bytes(32))]; resign(b)
    add(b.bincode(), 7, "include unknown authority")
    b = copy.deepcopy(base); b.includes = b.includes + [B.BlockReference(1, 2, bytes(32))]; resign(b)
    add(b.bincode(), 8, "include round == own round")
    b = copy.deepcopy(base); b.statements = [("range", base.includes[1], 5, 3)]; resign(b)
    add(b.bincode(), 9, "VoteRange end < start")
    b = copy.deepcopy(base); b.statements = [("range", base.includes[1], 0, 1 << 20)]; resign(b)
    add(b.bincode(), 11, "VoteRange too long")
    b = copy.deepcopy(base); b.statements = [("range", base.includes[1], 1, 1 << 20)]; resign(b)
    add(b.bincode(), 12, "VoteRange end too large")
    b = copy.deepcopy(base)
    b.statements = [("range", base.includes[1], 0, 7), ("range", base.includes[2], 2, 1 << 20),
                    ("range", base.includes[3], 5, 3)]
    resign(b)
    add(b.bincode(), 12, "VoteRange: the first failing range decides")
    b = copy.deepcopy(base)
    b.includes = b.includes + [B.BlockReference(1, 2, bytes(32)), B.BlockReference(9, 1, bytes(32))]
    resign(b)
    add(b.bincode(), 8, "includes: the first failing include decides")
    b = copy.deepcopy(base); b.includes = b.includes[:2]; resign(b)
    add(b.bincode(), 10, "threshold clock: 2 of 4 stake")
    b = copy.deepcopy(base)
    b.statements = [("share", b"hello"), ("accept", B.Locator(base.includes[1], 3)),
                    ("reject", B.Locator(base.includes[2], 4), None),
                    ("reject", B.Locator(base.includes[2], 5), B.Locator(base.includes[3], 6)),
                    ("range", base.includes[3], 1, 9)]
    resign(b)
    add(b.bincode(), 0, "all statement kinds")
    b = copy.deepcopy(base); b.epoch_marker = True; resign(b)
    add(b.bincode(), 0, "epoch marker set")
    b = copy.deepcopy(base); b.meta_creation_time_ns = 2**127 + 12345; resign(b)
    add(b.bincode(), 0, "u128 time high bits")
    raw = base.bincode()
    add(raw[:-1], 1, "truncated signature")
    add(raw[:100], 1, "truncated includes")
    add(raw + b"\x00\x01", 0, "trailing bytes (allowed by bincode::deserialize)")
    mark_pos = len(raw) - 64 - 8 - 8 - 1
    bad = bytearray(raw); bad[mark_pos] = 2
    add(bytes(bad), 1, "invalid bool epoch_marker")
    bad = bytearray(raw); bad[16] = 31
    add(bytes(bad), 1, "digest length 31")
    st = copy.deepcopy(base); st.statements = [("share", b"x")]; resign(st)
    sb = bytearray(st.bincode()); pos = 8 + 8 + 8 + 32 + 8 + 4 * 56 + 8
    sb[pos] = 3
    add(bytes(sb), 1, "invalid BaseStatement tag")
    return {"committee": committee_zero(4), "cases": cases}


def gen_block_zip215():
    """ZIP-215 signature edge cases inside whole StatementBlocks (crypto.rs:174-189: msg =
    Blake2b-256(pre-image), then VerificationKey::verify; types.rs:346-348: any error ->
    InvalidSignature, status 6). Every block passes the other checks, so its status is decided
    by the signature alone: 0 iff the pure-Python ZIP-215 predicate accepts.

    Committee: authorities 0..3 hold the zero-seed key with stake 100 each (their round-1
    blocks are every block's includes, so the threshold clock always passes); then every
    small-order encoding (canonical, y >= p, x = 0 with the sign bit set), a mixed-order key
    A + T for two torsion points T, a y >= p key that decodes to a point of unknown discrete
    log, and an undecodable key, stake 1 each."""
    import copy

    real_seed = B.ZERO_SEED
    real_pk = Z.public_key(real_seed)
    a_sc = Z._clamp(hashlib.sha512(real_seed).digest())
    A = Z.scalarmult(Z.B_POINT, a_sc)
    enc = Z.small_order_encodings()
    tors = [p for _, p in sorted(Z.torsion_points().items()) if not Z.is_identity(p)]
    keys, notes = [real_pk] * 4, ["zero-seed key"] * 4
    for e, canon in enc:
        keys.append(e)
        notes.append(f"small-order key ({'canonical' if canon else 'non-canonical'})")
    mixed_keys = []
    for ti in (0, 3):
        keys.append(Z.compress(Z.add(A, tors[ti])))
        notes.append(f"mixed-order key A + T{ti}")
        mixed_keys.append(len(keys) - 1)
    odd_y = None
    for y in range(2, 19):  # a y >= p encoding that decodes, not small order
        e = (y + Z.P).to_bytes(32, "little")
        pt = Z.decompress(e)
        if pt is not None and not Z.is_identity(Z.scalarmult(pt, 8)):
            odd_y = e
            break
    assert odd_y is not None
    keys.append(odd_y)
    notes.append("non-canonical key y >= p (decodes, unknown discrete log)")
    bad_key = None
    for y in range(2, 100):
        e = y.to_bytes(32, "little")
        if Z.decompress(e) is None:
            bad_key = e
            break
    keys.append(bad_key)
    notes.append("undecodable key")
    small_key_ids = [4 + i for i in range(len(enc))]
    stakes = [100] * 4 + [1] * (len(keys) - 4)

    r1 = B.gen_config1(Z.sign, rounds=1)  # round-1 blocks of authorities 0..3 (zero seed)
    incs = [b.reference() for b in r1]
    base = B.StatementBlock(0, 2, incs, [("share", b"zip215")], 2 * 10**8, False, 0)
    cases = []

    def add(author: int, make_sig, note: str):
        b = copy.deepcopy(base)
        b.authority = author
        b.meta_creation_time_ns = 2 * 10**8 + len(cases)  # every block distinct
        msg = b.signed_message()
        b.signature = make_sig(msg)
        b.digest = b.compute_digest()
        sig_st = Z.verify_status(keys[author], b.signature, msg)
        st = 0 if sig_st == Z.SIG_OK else 6
        cases.append({"bincode": b.bincode().hex(), "status": st, "msg_digest": msg.hex(),
                      "block_digest": b.digest.hex(), "note": f"{note} [author {author}: {notes[author]}]"})

    def ka_sig(R_enc: bytes, pk: bytes, msg: bytes) -> bytes:  # a signature with R of discrete log 0
        k = Z.sha512_mod_l(R_enc, pk, msg)
        return R_enc + (k * a_sc % Z.L).to_bytes(32, "little")

    # 1. small-order key x every small-order R encoding, s = 0: accepted (ZIP-215)
    for ai in small_key_ids:
        for r, canon in enc:
            add(ai, lambda m, r=r: r + bytes(32), f"small-order R ({'canonical' if canon else 'non-canonical'}), s = 0")
    # 2. small-order key, a real signature's R and s: rejected
    for ai in small_key_ids[:3]:
        add(ai, lambda m: Z.sign(real_seed, m), "real (R, s) under a small-order key")
    # 3. the real key: an honest signature, and R of discrete log 0 in every small-order encoding
    #    (identity / order-4 / order-2 points, canonical and non-canonical) with S = k a: the
    #    cofactored check accepts exactly those whose R is of order dividing 8
    add(0, lambda m: Z.sign(real_seed, m), "honest signature")
    for r, canon in enc:
        add(1, lambda m, r=r: ka_sig(r, real_pk, m), f"R small-order ({'canonical' if canon else 'non-canonical'}), S = k a")
    # 4. mixed-order R = rB + T with S re-derived: accepted (cofactored)
    for ti, T in enumerate(tors):
        def mixed_r(m, T=T, ti=ti):
            r = Z.sha512_mod_l(b"blk-mixed", bytes([ti]))
            Rb = Z.compress(Z.add(Z.scalarmult(Z.B_POINT, r), T))
            k = Z.sha512_mod_l(Rb, real_pk, m)
            return Rb + ((r + k * a_sc) % Z.L).to_bytes(32, "little")
        add(2, mixed_r, f"mixed-order R (torsion {ti}), S re-derived")
    # 5. mixed-order key A + T signed with a (k over the key's own encoding): accepted
    for ai in mixed_keys:
        def mixed_a(m, ai=ai):
            r = Z.sha512_mod_l(b"blk-mixedA", m)
            Rb = Z.compress(Z.scalarmult(Z.B_POINT, r))
            k = Z.sha512_mod_l(Rb, keys[ai], m)
            return Rb + ((r + k * a_sc) % Z.L).to_bytes(32, "little")
        add(ai, mixed_a, "signed with a under k(A + T)")
        add(ai, lambda m: Z.sign(real_seed, m), "RFC 8032 signature of A under A + T (k differs)")
    # 6. the y >= p key and the undecodable key
    oi, bi = len(keys) - 2, len(keys) - 1
    add(oi, lambda m: enc[0][0] + bytes(32), "small-order R, s = 0 under a y >= p key")
    add(oi, lambda m: Z.sign(real_seed, m), "real signature under a y >= p key")
    add(bi, lambda m: Z.sign(real_seed, m), "real signature under an undecodable key (MalformedPublicKey)")
    add(bi, lambda m: enc[0][0] + bytes(32), "small-order R, s = 0 under an undecodable key")
    # 7. s out of range and undecodable R for the real key
    for name, f in [("s = l", lambda s: Z.L), ("s + l", lambda s: s + Z.L), ("s = 2^255 - 1", lambda s: 2**255 - 1),
                    ("s high bit", lambda s: s | (1 << 255))]:
        def s_sig(m, f=f):
            sg = Z.sign(real_seed, m)
            return sg[:32] + f(int.from_bytes(sg[32:], "little")).to_bytes(32, "little")
        add(3, s_sig, name)
    add(3, lambda m: bad_key + Z.sign(real_seed, m)[32:], "R undecodable")
    add(3, lambda m: (Z.P + 3).to_bytes(32, "little") + Z.sign(real_seed, m)[32:], "R y >= p (y = 3)")
    add(0, lambda m: odd_y + bytes(32), "R y >= p of unknown discrete log, s = 0")
    add(0, lambda m: enc[0][0] + bytes(32), "R small-order, s = 0 under the real key")
    for bit in (0, 255, 256, 511):
        def flip(m, bit=bit):
            sg = bytearray(Z.sign(real_seed, m))
            sg[bit // 8] ^= 1 << (bit % 8)
            return bytes(sg)
        add(0, flip, f"signature bit {bit} flipped")
    return {
        "committee": {"pks": [k.hex() for k in keys], "stakes": stakes, "epoch": 0, "notes": notes},
        "round1_blocks": [b.bincode().hex() for b in r1],
        "accepted": sum(1 for c in cases if c["status"] == 0),
        "cases": cases,
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--skip-1m", action="store_true")
    ap.add_argument("--only", default="", help="regenerate one fixture file, e.g. block_edge.json")
    args = ap.parse_args()
    os.makedirs(GOLDEN, exist_ok=True)

    if args.only:
        gen = {"block_edge.json": gen_block_edge, "hash_kat.json": gen_hash_kat, "sig_kat.json": gen_sig_kat,
               "zip215_corpus.json": gen_zip215_corpus,
               "block_zip215.json": gen_block_zip215}[args.only]
        with open(os.path.join(GOLDEN, args.only), "w") as f:
            json.dump(gen(), f, indent=1)
        print("wrote", args.only)
        return

    def dump(name, obj):
        with open(os.path.join(GOLDEN, name), "w") as f:
            json.dump(obj, f, indent=1)
        print("wrote", name)

    dump("hash_kat.json", gen_hash_kat())
    dump("sig_kat.json", gen_sig_kat())
    dump("zip215_corpus.json", gen_zip215_corpus())
    dump("blocks_config1.json", gen_blocks_config1())
    dump("blocks_config4_sample.json", gen_blocks_config4_sample())
    dump("block_edge.json", gen_block_edge())
    dump("block_zip215.json", gen_block_zip215())
    if not args.skip_1m:
        spec, spec_c = gen_batch(1 << 20)
        dump("batch_config2.json", spec)
        dump("batch_config3.json", spec_c)


if __name__ == "__main__":
    main()
