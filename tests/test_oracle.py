"""CPU: pin the oracle (C restatement + Python ZIP-215 predicate) to the golden fixtures.

The fixtures come from independent sources (hashlib, libsodium RFC 8032, the
pure-Python predicate) — see oracle/gen_fixtures.py. Reference-side Rust parity
is unpinned (no cargo; the reference's tests stub crypto out, crypto.rs:63-75).
"""
import hashlib
import random
import struct

import numpy as np
import pytest

import blocks as B
import oracle as O
import zip215 as Z


def kat_input(n):
    return bytes((i * 31 + 7) % 251 for i in range(n))


def test_hash_kats(golden):
    g = golden("hash_kat.json")
    for n, d in g["blake2b256"].items():
        assert O.blake2b256(kat_input(int(n))).hex() == d, n
    for n, d in g["sha512"].items():
        assert O.sha512(kat_input(int(n))).hex() == d, n
    a0 = g["genesis_A0"]
    assert bytes.fromhex(a0["preimage_hex"]) == bytes(41)
    assert O.blake2b256(bytes(41)).hex() == a0["msg"]
    assert O.blake2b256(bytes(41 + 64)).hex() == a0["digest"]
    assert O.public_key(bytes(32)).hex() == g["zero_seed_pk"]


def test_sig_kats(golden):
    for c in golden("sig_kat.json"):
        seed, msg = bytes.fromhex(c["seed"]), bytes.fromhex(c["msg"])
        assert O.public_key(seed).hex() == c["pk"]
        assert O.sign(seed, msg).hex() == c["sig"]
        assert O.verify(bytes.fromhex(c["pk"]), bytes.fromhex(c["sig"]), msg) == O.SIG_OK


def test_zip215_corpus_c_oracle(golden):
    cases = golden("zip215_corpus.json")
    assert len(cases) > 230
    for c in cases:
        st = O.verify(bytes.fromhex(c["pk"]), bytes.fromhex(c["sig"]), bytes.fromhex(c["msg"]))
        assert st == c["status"], c["note"]


def test_zip215_corpus_has_all_verdict_kinds(golden):
    cases = golden("zip215_corpus.json")
    kinds = {c["status"] for c in cases}
    assert kinds == {0, 1, 2}
    assert sum(1 for c in cases if c["note"].endswith("s=0") and c["note"].startswith("small-order A")) == 196
    assert all(c["status"] == 0 for c in cases if c["note"].startswith("mixed-order"))


def test_python_predicate_matches_c_random():
    r = random.Random(7)
    for _ in range(40):
        seed = bytes(r.randrange(256) for _ in range(32))
        msg = bytes(r.randrange(256) for _ in range(32))
        pk, sig = O.public_key(seed), O.sign(seed, msg)
        bad = bytearray(sig)
        bad[r.randrange(64)] ^= 1 << r.randrange(8)
        for s in (sig, bytes(bad)):
            assert O.verify(pk, s, msg) == Z.verify_status(pk, s, msg)


def test_scalar_reduce_edges():
    for v in [0, 1, Z.L - 1, Z.L, Z.L + 1, 2 * Z.L, 2**512 - 1, 2**256, Z.L * Z.L]:
        assert O.scalar_reduce_wide(v.to_bytes(64, "little")) == (v % Z.L).to_bytes(32, "little")


def test_block_edge_statuses(golden):
    e = golden("block_edge.json")
    pks = np.frombuffer(b"".join(bytes.fromhex(x) for x in e["committee"]["pks"]), dtype=np.uint8).reshape(-1, 32)
    stakes = np.array(e["committee"]["stakes"], dtype=np.uint64)
    for c in e["cases"]:
        st, _, _ = O.block_verify(bytes.fromhex(c["bincode"]), pks, stakes, e["committee"]["epoch"])
        assert st == c["status"], c["note"]


def test_decoded_committee_path_matches(golden):
    """orc_committee (keys decoded once, the CPU baseline's form) gives the per-verify-decode
    path's statuses and digests on every edge case and on config-1 blocks, on 1 and 4 threads."""
    e = golden("block_edge.json")
    pks = np.frombuffer(b"".join(bytes.fromhex(x) for x in e["committee"]["pks"]), dtype=np.uint8).reshape(-1, 32)
    stakes = np.array(e["committee"]["stakes"], dtype=np.uint64)
    bins = [bytes.fromhex(c["bincode"]) for c in e["cases"]]
    buf = np.frombuffer(b"".join(bins) + b"\0", dtype=np.uint8)
    lens = np.array([len(x) for x in bins], dtype=np.uint64)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
    want = np.array([c["status"] for c in e["cases"]], dtype=np.uint8)
    for threads in (1, 4):
        a = O.block_verify_batch(buf, offs, lens, pks, stakes, e["committee"]["epoch"], threads)
        b = O.block_verify_batch(buf, offs, lens, pks, stakes, e["committee"]["epoch"], threads,
                                 decoded_committee=True)
        assert (a[0] == want).all() and (b[0] == want).all()
        assert (a[1] == b[1]).all() and (a[2] == b[2]).all()


def test_config1_blocks_oracle(golden):
    g = golden("blocks_config1.json")
    blks = B.gen_config1(O.sign)
    bins = [b.bincode() for b in blks]
    assert hashlib.sha256(b"".join(bins)).hexdigest() == g["sha256_bincode_concat"]
    for f, b in zip(g["first"], bins):
        assert b.hex() == f["bincode"]
        assert O.block_preimage(b).hex() == f["preimage"]
    buf = np.frombuffer(b"".join(bins), dtype=np.uint8)
    lens = np.array([len(x) for x in bins], dtype=np.uint64)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
    pks = np.frombuffer(b"".join(bytes.fromhex(x) for x in g["committee"]["pks"]), dtype=np.uint8).reshape(-1, 32)
    st, md, bd = O.block_verify_batch(buf, offs, lens, pks, np.ones(4, dtype=np.uint64), 0)
    assert (st == 0).all()
    assert hashlib.sha256(md.tobytes()).hexdigest() == g["sha256_msg_digests"]
    assert hashlib.sha256(bd.tobytes()).hexdigest() == g["sha256_block_digests"]


def test_config4_sample_oracle(golden):
    g = golden("blocks_config4_sample.json")
    blks = B.gen_config4(O.sign, rounds=2)
    bins = [b.bincode() for b in blks]
    assert len(bins[0]) == g["bincode_len_first"]
    assert hashlib.sha256(b"".join(bins)).hexdigest() == g["sha256_bincode_concat"]
    assert hashlib.sha256(b"".join(b.digest for b in blks)).hexdigest() == g["sha256_block_digests"]
    pks = np.frombuffer(b"".join(bytes.fromhex(x) for x in g["committee"]["pks"]), dtype=np.uint8).reshape(-1, 32)
    for b in bins[:5]:
        st, md, bd = O.block_verify(b, pks, np.ones(100, dtype=np.uint64), 0)
        assert st == 0


def test_batch_corpus_spec_prefix(golden):
    """The config-2/3 generator rules reproduce; a 2k prefix signs identically (full 1M runs on GPU)."""
    g = golden("batch_config3.json")
    n = 2048
    seeds = np.frombuffer(b"".join(hashlib.sha512(b"mysti-seed" + struct.pack("<Q", i)).digest()[:32]
                                   for i in range(n)), dtype=np.uint8).reshape(n, 32)
    msgs = np.frombuffer(b"".join(hashlib.blake2b(b"mysti-msg" + struct.pack("<Q", i), digest_size=32).digest()
                                  for i in range(n)), dtype=np.uint8).reshape(n, 32)
    pk, sig = O.sign_batch(seeds, msgs)
    st = O.verify_batch(pk, sig, msgs)
    assert (st == 0).all()
    for k, v in g["first_corrupted"].items():
        i = int(k)
        if i >= n:
            continue
        c = hashlib.sha256(b"mysti-corrupt" + struct.pack("<Q", i)).digest()
        bit = int.from_bytes(c[4:6], "little") % 512
        s = bytearray(sig[i].tobytes())
        s[bit // 8] ^= 1 << (bit % 8)
        assert O.verify(pk[i].tobytes(), bytes(s), msgs[i].tobytes()) == v
