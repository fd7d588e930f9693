"""GPU: the N > 1 path on the engine itself: two ranks (processes) with gloo
host collectives, both on device 0 of the one-GPU box, each verifying its own shard through
the C ABI -- signatures on the batch path and blocks through mv_verify_blocks -- with the
verdicts checked against the oracle and combined with all_ranks_ok, as bench.py does. The
shard is the verify loop of net_sync.rs:331-375; there is no exchange step, so no RCCL."""
import hashlib
import os
import struct

import numpy as np
import pytest
import torch.multiprocessing as mp

from mysticeti_amd.dist import all_ranks_ok, free_port, shard_range

pytestmark = pytest.mark.gpu

PER_RANK = 8192  # >= MV_BATCH_MIN: the batch path


def _worker(rank, world, port, out):
    import sys

    import torch.distributed as dist

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    sys.path.insert(0, os.path.join(root, "oracle"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import blocks as B
    import mysticeti_amd as M
    import oracle as O

    lo, hi = shard_range(rank, world, PER_RANK)
    seed = np.frombuffer(b"".join(hashlib.sha512(b"mysti-seed" + struct.pack("<Q", i)).digest()[:32]
                                  for i in range(lo, hi)), dtype=np.uint8).reshape(-1, 32)
    msg = np.frombuffer(b"".join(hashlib.blake2b(b"mysti-msg" + struct.pack("<Q", i), digest_size=32).digest()
                                 for i in range(lo, hi)), dtype=np.uint8).reshape(-1, 32)
    with M.Engine(devices=(0,)) as eng:
        pk, sig = eng.ed25519_sign(seed, msg)
        sig = sig.copy()
        bad = np.arange(rank + 5, PER_RANK, 977)  # a different bad set per rank
        sig[bad, 40] ^= 0x10
        st = eng.ed25519_verify(msg, sig, pk)
        want = np.zeros(PER_RANK, np.uint8)
        want[bad] = 1
        sample = np.arange(0, PER_RANK, 61)
        ok_sig = bool((st == want).all()) and bool((O.verify_batch(pk[sample], sig[sample], msg[sample]) == st[sample]).all())
        # blocks: each rank its own rounds of config-1 blocks, one block tampered per rank
        blks = B.gen_config1(O.sign, rounds=4 + rank)
        pks = np.frombuffer(O.public_key(bytes(32)) * 4, dtype=np.uint8).reshape(4, 32)
        eng.set_committee(pks, np.ones(4, dtype=np.uint64), 0)
        bins = [b.bincode() for b in blks]
        t = bytearray(bins[-1])
        t[-1] ^= 1  # a signature byte
        bins[-1] = bytes(t)
        bst, _, _ = eng.verify_blocks(bins)
        ost = np.array([O.block_verify(b, pks, np.ones(4, dtype=np.uint64), 0)[0] for b in bins], dtype=np.uint8)
        ok_blk = bool((bst == ost).all()) and int(bst[-1]) != 0 and bool((bst[:-1] == 0).all())
    out[rank] = (lo, hi, ok_sig, ok_blk, all_ranks_ok(ok_sig and ok_blk, dist))
    dist.destroy_process_group()


def test_two_ranks_on_the_engine():
    world = 2
    out = mp.Manager().dict()
    mp.spawn(_worker, args=(world, free_port(), out), nprocs=world, join=True)
    r0, r1 = out[0], out[1]
    assert (r0[0], r0[1]) == (0, PER_RANK) and (r1[0], r1[1]) == (PER_RANK, 2 * PER_RANK)
    assert r0[2] and r1[2], "a rank's signature verdicts differ from the oracle / the planted mask"
    assert r0[3] and r1[3], "a rank's block verdicts differ from the oracle"
    assert r0[4] and r1[4]
