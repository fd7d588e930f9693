"""WAL replay check throughput on an HBM-resident WAL image.

The image is what BlockStore::open replays (block_store.rs:66): WAL_ENTRY_BLOCK (tag 1) entries
whose payloads are config-4 StatementBlock bincode (4,100 distinct 100-validator blocks,
repeated), written with WalWriter's layout (16-MiB maps, wal.rs:95-188) and crc32 headers from
zlib (not from the library). One step = mv_dev_wal_verify over the whole image: the per-map
header walk, then the crc pass (one wave per entry), every entry checked.

Used by `bench.py --workload wal` and by the default bench line's "wal" key.
"""
from __future__ import annotations

import os
import struct
import time
import zlib

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
PEAK_HBM_BPS = 8.0e12  # MI355X HBM3E (MI355X_MICROARCH.md)
WAL_ENTRY_BLOCK = 1    # block_store.rs:496


def build_image(payloads, n: int, map_bits: int):
    """Host image of n entries cycling through `payloads`, WalWriter layout (the tests' size)."""
    import mysticeti_amd as M

    lens = np.array([len(payloads[i % len(payloads)]) for i in range(n)], dtype=np.uint64)
    pos, end = M.wal_layout(lens, map_bits)
    img = np.zeros(end + 16, dtype=np.uint8)
    hdrs = [struct.pack("<QII", zlib.crc32(p), len(p) + 16, WAL_ENTRY_BLOCK) for p in payloads]
    ents = [np.frombuffer(h + p, dtype=np.uint8) for h, p in zip(hdrs, payloads)]
    mv = img
    k = len(payloads)
    for i, p in enumerate(pos.tolist()):
        e = ents[i % k]
        mv[p:p + e.size] = e
    return img, pos, lens, end


def entry_runs(pos: np.ndarray, size: np.ndarray, k: int):
    """Maximal runs [a, b) of entries that lie back to back in the image AND in one cycle of the
    k distinct entries (so a run is one contiguous copy from the concatenated entries)."""
    n = pos.size
    nxt = np.ones(n, dtype=bool)  # entry i + 1 continues i's run
    nxt[:-1] = (pos[1:] == pos[:-1] + size[:-1]) & ((np.arange(1, n) % k) != 0)
    nxt[-1] = False
    ends = np.flatnonzero(~nxt) + 1
    starts = np.concatenate(([0], ends[:-1]))
    return starts, ends


def build_image_device(payloads, n: int, map_bits: int, torch, dev):
    """The same image built in HBM from the k distinct entries (a few hundred slice copies), so
    a rank holds ~40 MB of entries on the host instead of the whole ~10 GB image."""
    import mysticeti_amd as M

    k = len(payloads)
    lens = np.array([len(payloads[i % k]) for i in range(n)], dtype=np.uint64)
    pos, end = M.wal_layout(lens, map_bits)
    ents = b"".join(struct.pack("<QII", zlib.crc32(p), len(p) + 16, WAL_ENTRY_BLOCK) + p for p in payloads)
    ent_off = np.zeros(k + 1, dtype=np.int64)
    ent_off[1:] = np.cumsum([len(p) + 16 for p in payloads])
    d_ents = torch.from_numpy(np.frombuffer(ents, dtype=np.uint8).copy()).to(dev)
    img = torch.zeros(end + 16, dtype=torch.uint8, device=dev)
    size = lens.astype(np.int64) + 16
    starts, ends = entry_runs(pos.astype(np.int64), size, k)
    for a, b in zip(starts.tolist(), ends.tolist()):
        src0 = int(ent_off[a % k])
        nbytes = int(ent_off[(b - 1) % k + 1]) - src0
        dst0 = int(pos[a])
        img[dst0:dst0 + nbytes].copy_(d_ents[src0:src0 + nbytes])
    del d_ents
    return img, pos, lens, end


def cpu_baseline(img: np.ndarray, end: int, map_bits: int, seconds: float = 6.0, max_entries: int = 0) -> dict:
    """The oracle's WalIterator restatement (oracle/wal.c, crc32 by PCLMULQDQ folding as
    crc32fast does on x86_64), one thread as BlockStore::open replays, on a prefix sample."""
    import subprocess
    import ctypes
    import sys

    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "-s", "native"], check=True)
    lib = ctypes.CDLL(os.path.join(ROOT, "oracle", "build", "libmv_oracle_native.so"))
    vp = ctypes.c_void_p
    lib.orc_wal_iter.argtypes = [vp, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32, vp, vp, vp, vp,
                                 ctypes.c_uint64]
    lib.orc_wal_iter.restype = ctypes.c_uint64
    sample = min(end, 1 << 30)  # 1 GiB prefix (whole entries: the iteration stops at end_pos)
    cap = sample // 16 + 2  # entries are >= 16 B; a known entry count bounds the arrays tighter
    if max_entries:
        cap = min(cap, max_entries + 2)
    pos = np.zeros(cap, dtype=np.uint64)
    tag = np.zeros(cap, dtype=np.uint32)
    ln = np.zeros(cap, dtype=np.uint32)
    st = np.zeros(cap, dtype=np.uint8)
    done, ents, t0 = 0, 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        cnt = lib.orc_wal_iter(img.ctypes.data, img.size, sample, map_bits, pos.ctypes.data, tag.ctypes.data,
                               ln.ctypes.data, st.ctypes.data, cap)
        done += sample
        ents += int(cnt)
    dt = time.perf_counter() - t0
    ok = bool((st[:min(int(cnt), cap)] == 0).all())
    return {"value": round(done / dt / 1e9, 3), "unit": "GB/s", "cores": 1, "kind": "port",
            "entries_per_s": round(ents / dt, 1), "correct": ok,
            "sample": f"first {sample / 2**30:.2f} GiB of the image, iterated repeatedly for ~{seconds:.0f} s on one "
                      f"thread (BlockStore::open replays sequentially)",
            "impl": "oracle/wal.c WalIterator restatement; crc32 by PCLMULQDQ folding (crc32fast 1.3.2's x86_64 "
                    "path), gcc -O3 -march=native"}


def wal_measure(eng, torch, local_rank, world, dist, n: int, steps: int, warmup: int, cpu: bool = True,
                map_bits: int = 24) -> dict:
    import mysticeti_amd as M
    import mysticeti_amd.blocks as MB
    from mysticeti_amd.dist import all_ranks_ok, hbm_sample, timed_region

    dev = torch.device("cuda", local_rank)
    base = MB.config4(eng, rounds=41)  # 4,100 distinct config-4 blocks (signed on the GPU)
    payloads = [bytes(b) for b in base]
    t0 = time.perf_counter()
    d_img, pos, lens, end = build_image_device(payloads, n, map_bits, torch, dev)
    torch.cuda.synchronize(dev)
    build_s = time.perf_counter() - t0
    cap = n
    d_pos = torch.zeros(cap, dtype=torch.int64, device=dev)
    d_tag = torch.zeros(cap, dtype=torch.int32, device=dev)
    d_len = torch.zeros(cap, dtype=torch.int32, device=dev)
    d_st = torch.full((cap,), 255, dtype=torch.uint8, device=dev)
    stream = torch.cuda.Stream(dev)
    counts = []

    def step():
        counts.append(eng.dev_wal_verify(local_rank, d_img, end, end, map_bits, d_pos, d_tag, d_len, d_st, cap,
                                         stream.cuda_stream))

    for _ in range(warmup):
        step()
    torch.cuda.synchronize(dev)
    hbm_sample(torch, dev, "wal")
    elapsed = timed_region(step, steps, lambda: torch.cuda.synchronize(dev), dist)
    # stage events on a few more steps (kept out of `value`)
    eng.stage_times(reset=True)
    eng.set_stage_timing(True)
    for _ in range(3):
        step()
    torch.cuda.synchronize(dev)
    tot, calls = eng.stage_times()
    eng.set_stage_timing(False)
    stage_ms = {k: round(tot[k] / calls[k], 4) for k in ("wal_walk", "wal_crc") if calls[k]}
    ok = all(c == n for c in counts)
    ok &= bool((d_st.cpu().numpy() == 0).all())
    ok &= d_pos.cpu().numpy().astype(np.uint64).tolist() == pos.tolist()
    ok &= bool((d_len.cpu().numpy().astype(np.uint64) == lens).all())
    # a corrupted entry: the iteration stops there with CRC_MISMATCH (the reference's panic point)
    k = n // 3
    flip = int(pos[k]) + 16 + int(lens[k]) // 2
    d_img[flip] ^= 1
    c = eng.dev_wal_verify(local_rank, d_img, end, end, map_bits, d_pos, d_tag, d_len, d_st, cap, stream.cuda_stream)
    ok &= c == k + 1 and int(d_st[k].item()) == M.WAL_CRC_MISMATCH
    d_img[flip] ^= 1
    ok = all_ranks_ok(ok, dist)
    image_bytes = end
    entry_bytes = int(lens.sum()) + 16 * n  # what the crc pass reads: headers + payloads
    value = image_bytes * world * steps / elapsed
    crc_ms = stage_ms.get("wal_crc")
    roof = None
    if crc_ms:
        from bench import pmc_traffic

        traffic, tsrc = pmc_traffic("k_wal_crc", "wal")
        ach = entry_bytes / (crc_ms * 1e-3)
        roof = {"bound": "hbm", "kernel": "k_wal_crc", "kernel_ms": crc_ms, "achieved": round(ach / 1e9, 1),
                "peak": PEAK_HBM_BPS / 1e9, "unit": "GB/s", "frac": round(ach / PEAK_HBM_BPS, 4), "traffic": traffic,
                "traffic_source": tsrc,
                "bytes_per_launch": entry_bytes,
                "work": "every header (16 B) and payload byte read once per launch (SURVEY.md 8 f4: HBM-bound "
                        "checksum); the walk kernel re-reads the 16-B headers"}
    out = {"value": round(value / 1e9, 3), "unit": "GB/s (WAL bytes verified)",
           "entries_per_s": round(n * world * steps / elapsed, 1), "ms_per_step": round(elapsed / steps * 1e3, 4),
           "data": f"synthetic WAL: {n} WAL_ENTRY_BLOCK entries of config-4 block bincode ({len(payloads)} distinct), "
                   f"WalWriter layout, zlib crc32 headers; built in HBM from the distinct entries in {build_s:.1f} s",
           "config": {"workload": "f4: WAL replay check (WalIterator + crc32 of every entry), HBM-resident image",
                      "entries_per_gpu": n, "image_bytes": image_bytes, "map_bits": map_bits,
                      "parallelism": f"shard-per-gpu x{world} (one WAL image per rank), no collective"},
           "stage_ms": stage_ms, "roofline": roof, "correct": bool(ok)}
    if cpu and int(os.environ.get("RANK", "0")) == 0:
        # the CPU leg iterates the image's first GiB: copy that prefix (plus one entry's slack) back
        pre = min(end, 1 << 30)
        img = d_img[: min(end + 16, pre + (1 << 16))].cpu().numpy()
        out["cpu_baseline"] = cpu_baseline(img, pre, map_bits, max_entries=n)
        del img
        out["speedup_vs_cpu"] = round(value / world / 1e9 / out["cpu_baseline"]["value"], 1)
    del d_img
    torch.cuda.empty_cache()
    return out
