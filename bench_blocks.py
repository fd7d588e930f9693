"""Block-path benchmarks behind `bench.py --workload config4|config5` (BASELINE.json configs 4, 5).

config4  Throughput of whole-block verification (StatementBlock::verify, types.rs:315-376) on
         config-4-shaped blocks: 100-validator committee, 67 includes, one 512-B Share tx,
         66 VoteRanges (pre-image ~8,060 B, bincode ~9.5 KB). The bincode of `--batch` blocks
         per GPU is resident in HBM (a 4,100-block corpus signed on the GPU, replicated on the
         device); one step = one mv_dev_verify_blocks pass over it: device bincode parse ->
         pre-image -> 2 x BLAKE2b-256 (shared prefix) -> SHA-512 -> batch ZIP-215 verify ->
         verdicts. N > 1: one process per GPU, each with its own shard (weak scaling, no
         collective on the data path), as bench.py.
config5  Latency of 64-block batches (the online path: one message of blocks from the block
         handler, net_sync.rs:314-386): submit -> verdicts through mv_verify_blocks on host
         buffers (PCIe both ways), p50/p99 over --batches batches, for config-1 and config-4
         shaped blocks; beside the oracle's StatementBlock::verify on 1 host core (the
         reference's sequential loop) and on 16 host threads.
The CPU legs time oracle/block.c (the checker; -O3 -march=native on the box), the only use
of oracle/ here.
"""
from __future__ import annotations

import ctypes
import hashlib
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
METRIC = "verified StatementBlock sigs/sec (1/2/4/8 MI355X) vs host-core ed25519-consensus"
PEAK_VALU_OPS = 256 * 128 * 2.4e9  # full-rate 32-bit VALU lane-ops/s (bench.py)
W_BLAKE2B_OPS = 2688               # 32-bit ops per BLAKE2b compression

def _cpu_threads():
    sys.path.insert(0, ROOT)
    from mysticeti_amd.dist import cpu_share

    return cpu_share()


def _oracle_native():
    subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "-s", "native"], check=True)
    lib = ctypes.CDLL(os.path.join(ROOT, "oracle", "build", "libmv_oracle_native.so"))
    vp = ctypes.c_void_p
    lib.orc_block_verify_batch.argtypes = [vp, vp, vp, ctypes.c_size_t, vp, vp, ctypes.c_uint32, ctypes.c_uint64,
                                           vp, vp, vp, ctypes.c_int]
    lib.orc_block_verify_batch_c.argtypes = [vp, vp, vp, vp, ctypes.c_size_t, vp, vp, vp, ctypes.c_int]
    return lib


def _p(a):
    return ctypes.c_void_p(a.ctypes.data)


def _cpu_blocks(comm, buf, off, ln, threads):
    """oracle StatementBlock::verify of the blocks on `threads` host threads (committee keys
    decoded once: `comm` is a _Committee)."""
    st = np.zeros(off.shape[0], dtype=np.uint8)
    comm.lib.orc_block_verify_batch_c(comm.ptr, _p(buf), _p(off), _p(ln), off.shape[0], _p(st), None, None, threads)
    return st


def _host_cpu():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return ""


def _pct(lat, q):
    return round(float(np.percentile(np.asarray(lat) * 1e6, q)), 1)


def _lat_summary(lat):
    return {"p50_us": _pct(lat, 50), "p99_us": _pct(lat, 99), "mean_us": round(float(np.mean(lat)) * 1e6, 1),
            "batches": len(lat)}


def run(args) -> int:
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    # one GPU per rank; a rehearsal with more ranks than GPUs (e.g. 2 ranks on a 1-GPU box) shares
    # devices round-robin (device_count does not initialise the GPU)
    local_rank %= max(1, torch.cuda.device_count())

    dist = None
    if world > 1:
        import torch.distributed as dist

        from mysticeti_amd.dist import init_gloo

        init_gloo(dist)
    torch.cuda.set_device(local_rank)
    sys.path.insert(0, ROOT)
    import mysticeti_amd as M

    eng = M.Engine(devices=(local_rank,))
    if "MV_PREP_CHAIN" not in os.environ:
        eng.set_option("MV_PREP_CHAIN", 2)  # the steps' streams are this script's (bench.py main)
    try:
        if args.workload == "config5":
            return config5(args, eng, rank)
        if args.workload == "wal":
            import bench_wal

            res = bench_wal.wal_measure(eng, torch, local_rank, world, dist, n=args.wal_entries, steps=args.steps,
                                        warmup=args.warmup, cpu=args.cpu_sample > 0)
            if rank == 0:
                out = {"metric": "WAL replay check throughput (WalIterator + crc32 per entry)"}
                out.update(res)
                out["n_gpus"], out["steps"], out["warmup"] = world, args.steps, args.warmup
                out["higher_is_better"], out["scaling"], out["vs_baseline"], out["dtype"] = True, "weak", None, "u8"
                print(json.dumps(out), flush=True)
            return 0 if res["correct"] else 1
        return config4(args, eng, torch, local_rank, rank, world, dist)
    finally:
        eng.close()
        if dist:
            dist.destroy_process_group()


# ------------------------------------------------------------------ config 5 (latency)
def _native_driver():
    """bench_native/concurrent.c (built here with gcc): N pthreads calling a verify function."""
    src = os.path.join(ROOT, "bench_native", "concurrent.c")
    out_dir = os.path.join(ROOT, "bench_native", "build")
    so = os.path.join(out_dir, "libmv_conc.so")
    if not os.path.exists(so) or os.path.getmtime(so) < os.path.getmtime(src):
        os.makedirs(out_dir, exist_ok=True)
        subprocess.run(["gcc", "-O2", "-fPIC", "-shared", "-pthread", "-o", so, src], check=True)
    lib = ctypes.CDLL(so)
    vp, u32, u64 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64
    lib.mvb_concurrent.restype = u64
    lib.mvb_concurrent.argtypes = [ctypes.c_int, vp, vp, vp, vp, vp, u32, u32, ctypes.c_int, ctypes.c_int,
                                   ctypes.c_double, u64, vp, u64, ctypes.POINTER(ctypes.c_double),
                                   ctypes.POINTER(u64), ctypes.POINTER(u64)]
    return lib


class _Committee:
    """orc_committee of the native oracle: committee keys decoded once, as the reference's
    Committee holds them (committee.rs:83-87)."""

    def __init__(self, lib, pks, stakes):
        vp = ctypes.c_void_p
        lib.orc_committee_new.restype = vp
        lib.orc_committee_new.argtypes = [vp, vp, ctypes.c_uint32, ctypes.c_uint64]
        lib.orc_committee_free.argtypes = [vp]
        self.lib, self._pks, self._stakes = lib, np.ascontiguousarray(pks), np.ascontiguousarray(stakes)
        self.ptr = lib.orc_committee_new(_p(self._pks), _p(self._stakes), pks.shape[0], 0)
        self.fn = ctypes.cast(lib.orc_block_verify_batch_c, vp).value

    def close(self):
        if self.ptr:
            self.lib.orc_committee_free(self.ptr)
            self.ptr = None


def _drive(drv, kind, fn, ctx, packed, per_call, callers, inner_threads=1, seconds=0.0, max_calls=0):
    """One mvb_concurrent run: latency summary, blocks/s, and whether every block was accepted."""
    buf, off, ln = packed
    cap = max(1, int(max_calls * callers) if max_calls else int(callers * seconds * 40000) + 1024)
    lat = np.zeros(cap, dtype=np.float64)
    wall, bad, err = ctypes.c_double(), ctypes.c_uint64(), ctypes.c_uint64()
    calls = drv.mvb_concurrent(kind, fn, ctx, _p(buf), _p(off), _p(ln), off.shape[0], per_call, callers,
                               inner_threads, seconds, max_calls, _p(lat), cap, ctypes.byref(wall), ctypes.byref(bad),
                               ctypes.byref(err))
    r = _lat_summary(lat[:min(calls, cap)])
    r["blocks_per_s"] = round(calls * per_call / wall.value, 1)
    return r, bool(calls) and bad.value == 0 and err.value == 0


def config5_measure(eng, batches=10000, conc_seconds=3.0, cpu=True, callers=None, fanin_callers=99) -> dict:
    """Config 5 on this rank's GPU: for config-1 and config-4 shaped blocks,
      - 64-block calls of mv_verify_blocks one after another (host buffers, PCIe both ways):
        p50/p99 over `batches` calls, beside the oracle's StatementBlock::verify of the same
        64 blocks on one host core (the reference's sequential loop) and on the CPU share;
      - `callers` concurrent 1-block callers for `conc_seconds` (one tokio task per peer,
        net_sync.rs:214-221, 314-386): the GPU queue merges them; the CPU leg verifies each
        block on the caller's own core (no pool);
      - the same with `fanin_callers` callers (default 99 = committee - 1 of config 4's
        100-validator committee: process_blocks runs one task per peer, net_sync.rs:214-221,
        committee.rs:56-57); the CPU leg then runs 99 threads on the box's CPU share.
    Every caller is a pthread of bench_native/concurrent.c, so Python caps neither side."""
    import mysticeti_amd.blocks as MB

    drv = _native_driver()
    olib = _oracle_native() if cpu else None
    threads, share_src = _cpu_threads()
    callers = callers or threads
    mv_fn = ctypes.cast(eng.lib.mv_verify_blocks, ctypes.c_void_p).value
    out = {"unit": "us", "host_cpu": _host_cpu(), "cpu_threads": threads, "cpu_threads_source": share_src,
           "shapes": {}}
    ok = True
    shapes = [x for x in os.environ.get("MV_BENCH_C5_SHAPES", "config1,config4").split(",") if x]  # diagnostics
    for shape in shapes:
        if shape == "config1":
            blocks = MB.config1(eng, rounds=64)
            pks, stakes = MB.committee(eng, 4, distinct=False)
        else:
            blocks = MB.config4(eng, rounds=4)
            pks, stakes = MB.committee(eng, 100, distinct=True)
        eng.set_committee(pks, stakes, 0)
        nb = (len(blocks) // 64) * 64
        packed = MB.pack(blocks[:nb])
        res = {"bincode_bytes_per_block": int(packed[2].mean())}
        _drive(drv, 0, mv_fn, eng.ctx, packed, 64, 1, max_calls=max(8, nb // 64))  # warm-up
        o0 = eng.online_stats()
        res["gpu"], g = _drive(drv, 0, mv_fn, eng.ctx, packed, 64, 1, max_calls=batches)
        o1 = eng.online_stats()
        res["gpu"]["online_requests"], res["gpu"]["online_launches"] = o1[0] - o0[0], o1[1] - o0[1]
        ok &= g
        comm = _Committee(olib, pks, stakes) if olib is not None else None
        if comm is not None:
            n1 = 100 if shape == "config4" else 300
            res["cpu_1t"], c1 = _drive(drv, 1, comm.fn, comm.ptr, packed, 64, 1, inner_threads=1, max_calls=n1)
            _drive(drv, 1, comm.fn, comm.ptr, packed, 64, 1, inner_threads=threads, max_calls=50)  # pool up
            res[f"cpu_{threads}t"], c2 = _drive(drv, 1, comm.fn, comm.ptr, packed, 64, 1, inner_threads=threads,
                                                max_calls=max(200, batches // 4))
            ok &= c1 and c2
            res["cpu_p50_over_gpu_p50"] = {k: round(res[k]["p50_us"] / res["gpu"]["p50_us"], 3)
                                           for k in ("cpu_1t", f"cpu_{threads}t")}
        # concurrent 1-block callers: the CPU share's thread count, then the reference's fan-in
        legs = [("concurrent_1_block_callers", callers)]
        if fanin_callers and fanin_callers != callers:
            legs.append(("fan_in_callers", fanin_callers))
        for key, nc in legs:
            conc = {"callers": nc, "seconds": conc_seconds}
            q0, o0 = eng.queue_stats(), eng.online_stats()
            conc["gpu"], g = _drive(drv, 0, mv_fn, eng.ctx, packed, 1, nc, seconds=conc_seconds)
            q1, o1 = eng.queue_stats(), eng.online_stats()
            conc["gpu"]["queue_calls"] = q1[0] - q0[0]
            if q1[1] > q0[1]:
                conc["gpu"]["calls_per_device_pass"] = round((q1[0] - q0[0]) / (q1[1] - q0[1]), 2)
            conc["gpu"]["online_requests"], conc["gpu"]["online_launches"] = o1[0] - o0[0], o1[1] - o0[1]
            ok &= g
            if comm is not None:
                conc["cpu_own_core"], c = _drive(drv, 1, comm.fn, comm.ptr, packed, 1, nc, inner_threads=1,
                                                 seconds=conc_seconds)
                ok &= c
                conc["gpu_over_cpu_blocks_per_s"] = round(
                    conc["gpu"]["blocks_per_s"] / conc["cpu_own_core"]["blocks_per_s"], 3)
            res[key] = conc
        if comm is not None:
            comm.close()
        out["shapes"][shape] = res
    out["correct"] = bool(ok)
    out["note"] = ("GPU: mv_verify_blocks on host buffers (raw bincode in, verdicts out; 64 blocks < MV_BATCH_MIN "
                   "take the committee comb tables, comb.hip); CPU: oracle/block.c StatementBlock::verify with the "
                   "committee keys decoded once (orc_committee), 64-block calls on 1 core and on the pooled CPU "
                   "share, concurrent callers each on its own core; every caller is a pthread "
                   "(bench_native/concurrent.c)")
    return out


def config5(args, eng, rank) -> int:
    res = config5_measure(eng, batches=args.batches, conc_seconds=args.conc_seconds, cpu=args.cpu_sample > 0,
                          fanin_callers=args.fanin_callers, callers=args.conc_callers or None)
    out = {"metric": "config5: 64-block batch verify latency, submit -> verdicts (mv_verify_blocks, host buffers)",
           "higher_is_better": False, "n_gpus": 1, "data": "synthetic (blocks signed on the GPU)"}
    out.update(res)
    if rank == 0:
        print(json.dumps(out), flush=True)
    return 0 if res["correct"] else 1


# ------------------------------------------------------------------ config 4 (throughput)
def config4(args, eng, torch, local_rank, rank, world, dist) -> int:
    res = config4_measure(eng, torch, local_rank, world, dist, n=args.batch, steps=args.steps, warmup=args.warmup,
                          nstreams=max(1, args.streams), cpu=args.cpu_sample > 0, host_blocks=args.host_fed_blocks)
    if rank == 0:
        out = {"metric": METRIC}
        out.update(res)
        out["n_gpus"] = world
        out["steps"], out["warmup"] = args.steps, args.warmup
        out["higher_is_better"], out["scaling"], out["vs_baseline"], out["dtype"] = True, "weak", None, "u32"
        print(json.dumps(out), flush=True)
    return 0 if res["correct"] else 1


def config4_host_fed(eng, torch, dev, buf, off, ln, nb, span, n_host, calls=3) -> dict:
    """Config 4 fed from host memory (PCIe-inclusive, BASELINE.md 3 row 4 "streamed in chunks"):
    `n_host` config-4 blocks in one pageable host buffer through mv_verify_blocks, which packs
    them into pinned staging in chunks and overlaps chunk c + 1's pack and H2D with chunk c's
    device pipeline. Best of `calls` calls. Beside it the measured pinned H2D bandwidth and the
    bound it sets: H2D GB/s / bincode bytes per block."""
    reps = (n_host + nb - 1) // nb
    base_bytes = int(off[-1] + ln[-1])
    hoff = (np.arange(reps, dtype=np.uint64)[:, None] * np.uint64(span) + off.astype(np.uint64)[None, :]).reshape(-1)[:n_host]
    hlen = np.tile(ln.astype(np.uint64), reps)[:n_host]

    def fill(b):  # the corpus repeated `reps` times, at the same offsets in either buffer
        b[reps * span:] = 0
        rows = b[: reps * span].reshape(reps, span)
        rows[:, :base_bytes] = buf[:base_bytes]
        rows[:, base_bytes:] = 0

    def best_of(b):
        eng.verify_blocks_packed(b, hoff[:nb].copy(), hlen[:nb].copy())  # warm the staging
        st_, best_ = None, None
        for _ in range(calls):
            t0 = time.perf_counter()
            st_, _, _ = eng.verify_blocks_packed(b, hoff, hlen)
            dt = time.perf_counter() - t0
            best_ = dt if best_ is None else min(best_, dt)
        return best_, st_

    # page-locked caller memory (mv_host_alloc): the engine DMAs the bytes in place; then the
    # same bytes in a pageable buffer (one of the two lives at a time: host RSS per rank)
    pbuf = eng.host_empty((reps * span + 64,))
    fill(pbuf)
    best, st = best_of(pbuf)
    eng.host_free(pbuf)
    del pbuf
    hbuf = np.empty(reps * span + 64, dtype=np.uint8)
    fill(hbuf)
    best_page, st_page = best_of(hbuf)
    del hbuf
    # pinned H2D bandwidth (256 MiB = the engine's chunk, torch's pinned allocator, the copy engine alone)
    h = torch.empty(256 << 20, dtype=torch.uint8).pin_memory()
    d = torch.empty(256 << 20, dtype=torch.uint8, device=dev)
    d.copy_(h, non_blocking=True)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(8):
        d.copy_(h, non_blocking=True)
    torch.cuda.synchronize(dev)
    h2d = 8 * (256 << 20) / (time.perf_counter() - t0)
    del h, d
    L = float(np.mean(hlen))
    rate = n_host / best
    return {"value": round(rate, 1), "unit": "blocks/s", "blocks": n_host,
            "bincode_GB": round(float(hlen.sum()) / 1e9, 3), "seconds": round(best, 4),
            "h2d_GBps_pinned": round(h2d / 1e9, 1), "pcie_bound_blocks_per_s": round(h2d / L, 1),
            "frac_of_pcie_bound": round(rate / (h2d / L), 4),
            "pageable": round(n_host / best_page, 1),
            "correct": bool((st == 0).all()) and bool((st_page == 0).all()),
            "note": "mv_verify_blocks over one host buffer of packed blocks, best of "
                    f"{calls} calls; value: the buffer in page-locked memory (mv_host_alloc), which the engine "
                    "DMAs in place in 256-MiB chunks (chunk c+1 copied while chunk c runs); pageable: a plain "
                    "numpy buffer, which the engine first packs into its pinned staging with 8 threads; the "
                    f"PCIe bound is the measured pinned H2D rate over {L:.0f} B per block"}


def config4_measure(eng, torch, local_rank, world, dist, n, steps, warmup, nstreams=2, cpu=True,
                    host_blocks=1 << 18) -> dict:
    """Config 4 on this rank's GPU: `n` HBM-resident config-4 blocks per step through
    mv_dev_verify_blocks (device parse -> pre-image -> 2 x BLAKE2b -> batch ZIP-215 -> verdicts);
    value = blocks/s over all ranks (weak scaling). Used by `--workload config4` and by the
    default bench.py line (its "config4" key)."""
    import mysticeti_amd as M
    import mysticeti_amd.blocks as MB
    from mysticeti_amd.dist import all_ranks_ok, hbm_sample, timed_region

    dev = torch.device("cuda", local_rank)
    rounds = 41
    base = MB.config4(eng, rounds=rounds)  # 4,100 distinct blocks
    pks, stakes = MB.committee(eng, 100, distinct=True)
    eng.set_committee(pks, stakes, 0)
    buf, off, ln = MB.pack(base)
    nb = len(base)
    base_bytes = int(off[-1] + ln[-1])
    span = (base_bytes + 7) & ~7
    reps = (n + nb - 1) // nb
    host = np.zeros(span, dtype=np.uint8)
    host[:base_bytes] = buf[:base_bytes]
    d_base = torch.from_numpy(host).to(dev)
    d_buf = torch.zeros(reps * span + 64, dtype=torch.uint8, device=dev)
    d_buf[: reps * span].view(reps, span).copy_(d_base.unsqueeze(0).expand(reps, span))
    off_all = (np.arange(reps, dtype=np.int64)[:, None] * span + off.astype(np.int64)[None, :]).reshape(-1)[:n]
    len_all = np.tile(ln.astype(np.int64), reps)[:n]
    d_off = torch.from_numpy(off_all).to(dev)
    d_len = torch.from_numpy(len_all).to(dev)
    buf_bytes = reps * span
    # Steps alternate over `nstreams` streams: the engine's two-slot block scratch ring orders
    # reuse, and one step's HBM-bound ingest and latency-bound batch tail (reduce, final)
    # overlap the other step's VALU-bound kernels. Stage times for the roofline are re-taken
    # on ONE stream after the timed region, so they match rocprofv3.
    streams = [torch.cuda.Stream(dev) for _ in range(nstreams)]
    d_st = [torch.full((n,), 255, dtype=torch.uint8, device=dev) for _ in range(nstreams)]
    d_md = [torch.zeros((n, 32), dtype=torch.uint8, device=dev) for _ in range(nstreams)]
    d_bd = [torch.zeros((n, 32), dtype=torch.uint8, device=dev) for _ in range(nstreams)]
    torch.cuda.synchronize(dev)
    state = {"i": 0}

    def step():
        j = state["i"] % nstreams
        state["i"] += 1
        eng.dev_verify_blocks(local_rank, d_buf, buf_bytes, d_off, d_len, d_st[j], d_md[j], d_bd[j],
                              streams[j].cuda_stream)

    for _ in range(warmup):
        step()
    torch.cuda.synchronize(dev)
    hbm_sample(torch, dev, "config4")
    # per-step record of the timed steps: host enqueue time and device time (a HIP event pair
    # on the step's stream), so a one-time cost inside the timed region shows in the line
    marks = []

    def timed_step():
        j = state["i"] % nstreams
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record(streams[j])
        step()
        e1.record(streams[j])
        marks.append((time.perf_counter() - t0, e0, e1))

    elapsed = timed_region(timed_step, steps, lambda: torch.cuda.synchronize(dev), dist)
    host_ms = [m[0] * 1e3 for m in marks]
    dev_ms = [m[1].elapsed_time(m[2]) for m in marks]
    summ = lambda v: {"first": round(v[0], 3), "median": round(float(np.median(v)), 3), "max": round(max(v), 3)}
    step_ms = {"device": summ(dev_ms), "host_enqueue": summ(host_ms),
               "note": "per timed step: device = HIP events around the call on its stream (steps on two "
                       "streams overlap, so these exceed ms_per_step); host_enqueue = the call's host time"}
    # the as-run stage table: stage events on a few more alternating steps (kept out of `value`)
    eng.stage_times(reset=True)
    eng.set_stage_timing(True)
    for _ in range(max(2 * nstreams, min(steps, 6))):
        step()
    torch.cuda.synchronize(dev)
    tot, calls = eng.stage_times()
    eng.set_stage_timing(False)
    stage_ms = {k: round(v / calls[k], 4) for k, v in tot.items() if calls[k]}
    stage_ms_run = stage_ms
    if nstreams > 1:
        eng.stage_times(reset=True)
        eng.set_stage_timing(True)
        for _ in range(3):
            eng.dev_verify_blocks(local_rank, d_buf, buf_bytes, d_off, d_len, d_st[0], d_md[0], d_bd[0],
                                  streams[0].cuda_stream)
        torch.cuda.synchronize(dev)
        tot, calls = eng.stage_times()
        eng.set_stage_timing(False)
        stage_ms = {k: round(v / calls[k], 4) for k, v in tot.items() if calls[k]}
    ok = all(bool((x.cpu().numpy() == 0).all()) for x in d_st)
    # block digests = the digests the blocks claim (bincode bytes 24..56), bit-exact
    bd = d_bd[0][:nb].cpu().numpy()
    claimed = np.stack([np.frombuffer(b[24:56], dtype=np.uint8) for b in base])
    ok &= bool((bd == claimed).all())
    msg_sha = hashlib.sha256(d_md[0][:nb].cpu().numpy().tobytes()).hexdigest()
    value = n * world * steps / elapsed
    L = int(np.mean([len(b) for b in base]))  # bincode length
    pre_len = len(M.block_preimage(base[0]))  # the host codec (block_codec.cpp)
    # shared prefix: (L-1)//128 compressions, then 1 final for B2(P) and the rest of B2(P || sig)
    comp_exec = (pre_len + 64 - 1) // 128 + 2
    comp_alg = -(-pre_len // 128) + -(-(pre_len + 64) // 128)
    hash_ms = stage_ms.get("hash")
    cpu_res = None
    if cpu and int(os.environ.get("RANK", "0")) == 0:  # the CPU baseline: rank 0 (bench.py asks at N = 1 only)
        lib = _oracle_native()
        comm = _Committee(lib, pks, stakes)
        threads, share_src = _cpu_threads()
        res = {}
        for t, seconds in ((1, 4.0), (threads, 8.0)):
            done, t0 = 0, time.perf_counter()
            sub = nb if t > 1 else 400
            o2, l2 = off[:sub].copy(), ln[:sub].copy()
            while time.perf_counter() - t0 < seconds:
                st = _cpu_blocks(comm, buf, o2, l2, t)
                ok &= bool((st == 0).all())
                done += sub
            res[t] = (done / (time.perf_counter() - t0), done)
        comm.close()
        cpu_res = {"value": round(res[threads][0], 1), "unit": "blocks/s", "cores": threads, "kind": "port",
                   "sample": f"{res[threads][1]} config-4 blocks on {threads} threads (~8 s); single core: "
                             f"{res[1][1]} blocks (~4 s)", "single_core_value": round(res[1][0], 1),
                   "host_cpu": _host_cpu(), "nproc": os.cpu_count(), "cores_source": share_src,
                   "impl": "oracle/block.c StatementBlock::verify (parse, 2 x BLAKE2b, ZIP-215 verify; committee keys "
                           "decoded once), gcc -O3 -march=native, persistent thread pool"}
    roof = None
    from bench import pmc_traffic

    # the dominant kernel: by default the one-pass walk (block_walk.hip, the "parse" stage: parse,
    # checks and both digests); MV_BLK_WALK=0: the staged form's hash (k_b2_lane, or k_b2_quad
    # with MV_B2_LANE=0)
    if os.environ.get("MV_BLK_WALK", "1").startswith("0"):
        kname = "k_b2_quad" if os.environ.get("MV_B2_LANE") == "0" else "k_b2_lane"
    else:
        kname, hash_ms = "k_block_walk", stage_ms.get("parse")
    traffic, traffic_src = pmc_traffic(kname, "c4")
    if hash_ms:
        ach = n * comp_exec * W_BLAKE2B_OPS / (hash_ms * 1e-3)
        # kernel_ms is one launch over the call's n blocks (stage timing runs it as one launch);
        # the PMC pass (tools/gpu.sh pmc:c4s1) launches it over 2^20 blocks, so its bytes are
        # scaled to n: both numbers are per the same n blocks
        traffic_n = round(traffic * n / (1 << 20)) if traffic else None
        roof = {"bound": "valu", "kernel": kname, "kernel_ms": hash_ms,
                "achieved": round(ach / 1e12, 3), "peak": round(PEAK_VALU_OPS / 1e12, 2), "unit": "TOP/s",
                "frac": round(ach / PEAK_VALU_OPS, 4), "traffic": traffic_n,
                "per": f"one launch over {n} blocks (kernel_ms, traffic, achieved)",
                "traffic_per_2^20_blocks": traffic, "traffic_source": traffic_src,
                "traffic_over_bincode": round(traffic / ((1 << 20) * L), 3) if traffic else None,
                "bincode_GBps": round(n * L / (hash_ms * 1e-3) / 1e9, 1),
                "work_per_block": f"{comp_exec} BLAKE2b compressions executed (shared prefix; {comp_alg} "
                                  f"algorithmic) x {W_BLAKE2B_OPS} ops; the transcode and checks are not "
                                  f"counted"}
    host_fed = None
    if int(os.environ.get("RANK", "0")) == 0 and host_blocks > 0:
        host_fed = config4_host_fed(eng, torch, dev, buf, off, ln, nb, span, host_blocks)
        ok &= host_fed["correct"]
    ok = all_ranks_ok(ok, dist)
    out = {"value": round(value, 1), "unit": "blocks/s (= verified block signatures/s)",
           "ms_per_step": round(elapsed / steps * 1e3, 4), "steps": steps, "warmup": warmup, "step_ms": step_ms,
           "data": f"synthetic config-4 blocks ({nb} distinct, signed on the GPU, replicated in HBM)",
           "config": {"workload": "config4: 100-validator blocks, 67 includes, 512-B tx, 66 VoteRanges, "
                                  "HBM-resident bincode, device parse + verify", "blocks_per_gpu": n,
                      "global_blocks": n * world,
                      "bincode_bytes_per_block": L, "preimage_bytes": pre_len,
                      "parallelism": f"shard-per-gpu x{world}, no collective"},
           "roofline": roof,
           "pipeline": {"stage_ms": stage_ms, "streams": nstreams,
                        "stage_ms_as_run": stage_ms_run if nstreams > 1 else None,
                        "note": "stage_ms: 3 post-run steps on one stream (roofline); "
                                "stage_ms_as_run: HIP events with overlapping streams",
                        "hbm_bincode_GBps": round(n * L / (elapsed / steps) / 1e9, 1)},
           "cpu_baseline": cpu_res, "host_fed": host_fed, "correct": bool(ok),
           "sha256_msg_digests_first_corpus": msg_sha}
    if cpu_res:
        out["speedup_vs_cpu"] = {"all_cores": round(value / world / cpu_res["value"], 1),
                                 "single_core": round(value / world / cpu_res["single_core_value"], 1)}
    del d_buf, d_st, d_md, d_bd
    return out
