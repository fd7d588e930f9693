"""Multi-GPU plumbing for bench.py: one process per GPU, no data-path collective.

Verification shards by independent signatures: rank r verifies the
corpus slice [r*n, (r+1)*n) on its own device, weak scaling. The only collectives
are host-side gloo ones around the timed region (barrier, max of the elapsed time,
sum of failure flags); no RCCL/xGMI traffic is needed and none is invented.
"""
from __future__ import annotations

import time
from typing import Callable, Optional, Tuple


def init_gloo(dist) -> None:
    """dist.init_process_group("gloo") with the C++ library's stdout chatter ("[Gloo] Rank r is
    connected to ...") sent to stderr: stdout carries only rank 0's JSON line."""
    import os
    import sys

    sys.stdout.flush()
    saved = os.dup(1)
    try:
        os.dup2(2, 1)
        dist.init_process_group("gloo")
    finally:
        sys.stdout.flush()
        os.dup2(saved, 1)
        os.close(saved)


def needs_launch(gpus: int, env=None) -> bool:
    """True when `--gpus N` (N > 1) was asked for but this process is not a rank of a launched
    job (no WORLD_SIZE): the bench must start its N ranks itself."""
    import os

    env = os.environ if env is None else env
    return gpus > 1 and "WORLD_SIZE" not in env


def free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(script: str, argv, nproc: int, timeout: Optional[float] = None) -> int:
    """Runs `script argv` as `nproc` ranks under torch.distributed.run (one process per GPU,
    rendezvous on 127.0.0.1) as a CHILD process and returns its exit code. The caller must not
    have touched the GPU: the ranks own the devices. stdout/stderr are inherited, so rank 0's
    JSON line (the only stdout line: gloo's chatter goes to stderr, init_gloo) reaches the
    caller's stdout as it is printed."""
    import subprocess
    import sys

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), script] + list(argv)
    sys.stdout.flush()
    sys.stderr.flush()
    return subprocess.run(cmd, timeout=timeout).returncode


def shard_range(rank: int, world: int, per_rank: int) -> Tuple[int, int]:
    """Corpus indices owned by `rank` (weak scaling: `per_rank` items each)."""
    assert 0 <= rank < world and per_rank >= 0
    return rank * per_rank, (rank + 1) * per_rank


def timed_region(step: Callable[[], None], steps: int, sync: Callable[[], None], dist=None) -> float:
    """Barrier + sync, run `steps` steps, sync + barrier; return the MAX elapsed over ranks."""
    sync()
    if dist is not None:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    return max_over_ranks(elapsed, dist)


def max_over_ranks(x: float, dist=None) -> float:
    if dist is None:
        return x
    import torch

    t = torch.tensor([x], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def all_ranks_ok(ok: bool, dist=None) -> bool:
    if dist is None:
        return ok
    import torch

    t = torch.tensor([0 if ok else 1], dtype=torch.int64)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return int(t.item()) == 0


def cpu_share() -> Tuple[int, str]:
    """Host cores this process may use: min of the CPU affinity mask, the cgroup v2/v1 CPU
    quota and OMP_NUM_THREADS (the GPU box exports its share there); with the source."""
    import os

    cores, src = os.cpu_count() or 1, "os.cpu_count"
    try:
        a = len(os.sched_getaffinity(0))
        if a < cores:
            cores, src = a, "sched_getaffinity"
    except (AttributeError, OSError):
        pass
    quota = None
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(p)
    except (OSError, ValueError):
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            p = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = q / p
        except (OSError, ValueError):
            pass
    if quota is not None and int(quota) < cores:
        cores, src = max(1, int(quota)), "cgroup cpu quota"
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and 0 < int(omp) < cores:
        cores, src = int(omp), "OMP_NUM_THREADS"
    return cores, src


# ---- per-rank footprint (host RSS, HBM) reported in the bench line
_hbm_peak = {"bytes": 0, "where": ""}
_rss_marks = []  # (leg, peak host RSS so far, GB): which leg raised the peak


def _maxrss_gb() -> float:
    import resource

    return round(resource.getrusage(resource.RUSAGE_SELF).ru_maxrss * 1024 / 1e9, 3)


def rss_mark(where: str) -> None:
    """Records the peak host RSS so far, after leg `where` (ru_maxrss only grows)."""
    _rss_marks.append((where, _maxrss_gb()))


def hbm_sample(torch, dev, where: str = "") -> None:
    """Records the device's HBM in use now (total - free, hipMemGetInfo) if it is the largest
    seen; call it where the bench holds the most (after each leg's buffers are live)."""
    free, total = torch.cuda.mem_get_info(dev)
    used = int(total - free)
    if used > _hbm_peak["bytes"]:
        _hbm_peak["bytes"], _hbm_peak["where"] = used, where


def footprint(rank: int, dist=None):
    """[{rank, host_rss_peak_GB, hbm_peak_GB, hbm_peak_at}] over all ranks (gloo all_gather of
    small dicts; rank order)."""
    me = {"rank": rank, "host_rss_peak_GB": _maxrss_gb(),
          "hbm_peak_GB": round(_hbm_peak["bytes"] / 1e9, 2), "hbm_peak_at": _hbm_peak["where"],
          "rss_after": dict(_rss_marks)}
    if dist is None:
        return [me]
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, me)
    return out
