"""CPU: the N>1 bench path (one process per GPU, gloo host collectives only) with
world_size 2 on the CPU: disjoint weak-scaling shards, max-over-ranks timing, and
per-rank verification of its own corpus slice (checked by the oracle)."""
import hashlib
import os
import struct

import numpy as np
import pytest
import torch.multiprocessing as mp

from mysticeti_amd.dist import all_ranks_ok, shard_range, timed_region


def _worker(rank, world, port, out):
    import time

    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import oracle as O

    lo, hi = shard_range(rank, world, 64)
    seed = np.frombuffer(b"".join(hashlib.sha512(b"mysti-seed" + struct.pack("<Q", i)).digest()[:32]
                                  for i in range(lo, hi)), dtype=np.uint8).reshape(-1, 32)
    msg = np.frombuffer(b"".join(hashlib.blake2b(b"mysti-msg" + struct.pack("<Q", i), digest_size=32).digest()
                                 for i in range(lo, hi)), dtype=np.uint8).reshape(-1, 32)
    pk, sig = O.sign_batch(seed, msg, 1)
    ok = bool((O.verify_batch(pk, sig, msg, 1) == 0).all())
    # rank 1 is deliberately slower: the reported time must be the max over ranks
    el = timed_region(lambda: time.sleep(0.05 * (rank + 1)), 2, lambda: None, dist)
    out[rank] = (lo, hi, el, all_ranks_ok(ok, dist), all_ranks_ok(rank == 0, dist))
    dist.destroy_process_group()


def test_two_rank_gloo():
    world = 2
    port = 29500 + os.getpid() % 1000
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, port, out), nprocs=world, join=True)
    r0, r1 = out[0], out[1]
    assert (r0[0], r0[1]) == (0, 64) and (r1[0], r1[1]) == (64, 128)
    assert r0[2] == r1[2] and r0[2] >= 0.2  # both report the slower rank's time
    assert r0[3] and r1[3]  # every shard verified
    assert not r0[4] and not r1[4]  # one failing rank fails the job


def test_shard_ranges_cover_without_overlap():
    for world in (1, 2, 4, 8):
        seen = []
        for r in range(world):
            lo, hi = shard_range(r, world, 1000)
            seen.extend(range(lo, hi))
        assert seen == list(range(world * 1000))


def test_torchrun_stdout_is_one_json_line(tmp_path):
    """bench.py's launch shape (torch.distributed.run, 2 ranks, gloo): the gloo library's own
    stdout chatter goes to stderr during init (init_gloo), so stdout holds only rank 0's line."""
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    script = tmp_path / "line.py"
    script.write_text(
        "import json, os, sys\n"
        f"sys.path.insert(0, {root!r})\n"
        "import torch.distributed as dist\n"
        "from mysticeti_amd.dist import all_ranks_ok, init_gloo\n"
        "init_gloo(dist)\n"
        "ok = all_ranks_ok(True, dist)\n"
        "if dist.get_rank() == 0:\n"
        "    print(json.dumps({'world': dist.get_world_size(), 'ok': ok}), flush=True)\n"
        "dist.destroy_process_group()\n")
    port = 29000 + os.getpid() % 900
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), str(script)],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, r.stdout
    assert json.loads(lines[0]) == {"world": 2, "ok": True}


def test_needs_launch():
    from mysticeti_amd.dist import needs_launch

    assert not needs_launch(1, {})
    assert needs_launch(2, {})
    assert not needs_launch(8, {"WORLD_SIZE": "8"})


def test_launch_ranks_starts_n_ranks_and_relays_rank0_line(tmp_path):
    """bench.py --gpus N without an external launcher: dist.launch_ranks starts N ranks of the
    script as a child torch.distributed.run (argv passed through) and returns its exit code;
    the caller's stdout gets exactly rank 0's JSON line."""
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    stub = tmp_path / "stub.py"
    stub.write_text(
        "import json, os, sys\n"
        f"sys.path.insert(0, {root!r})\n"
        "import torch.distributed as dist\n"
        "from mysticeti_amd.dist import all_ranks_ok, init_gloo\n"
        "init_gloo(dist)\n"
        "ok = all_ranks_ok(True, dist)\n"
        "if dist.get_rank() == 0:\n"
        "    print(json.dumps({'n_gpus': dist.get_world_size(), 'argv': sys.argv[1:], 'ok': ok}), flush=True)\n"
        "dist.destroy_process_group()\n"
        "sys.exit(3 if '--fail' in sys.argv else 0)\n")
    parent = tmp_path / "parent.py"
    parent.write_text(
        "import sys\n"
        f"sys.path.insert(0, {root!r})\n"
        "from mysticeti_amd.dist import launch_ranks, needs_launch\n"
        "n = int(sys.argv[1])\n"
        "assert needs_launch(n)\n"
        f"sys.exit(launch_ranks({str(stub)!r}, ['--gpus', str(n)] + sys.argv[2:], n))\n")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, str(parent), "2", "--steps", "3"], capture_output=True, text=True,
                       timeout=180, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, r.stdout
    assert json.loads(lines[0]) == {"n_gpus": 2, "argv": ["--gpus", "2", "--steps", "3"], "ok": True}
    r = subprocess.run([sys.executable, str(parent), "2", "--fail"], capture_output=True, text=True,
                       timeout=180, env=env)
    assert r.returncode != 0


def test_bench_refuses_a_world_that_differs_from_gpus():
    """A launched rank whose WORLD_SIZE differs from --gpus stops before touching a device."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "4"], capture_output=True,
                       text=True, timeout=120, env=env)
    assert r.returncode != 0 and "WORLD_SIZE=2" in r.stderr
