"""Benchmark: verified StatementBlock signatures / s on 1..8 MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[1], "config 2"): per GPU, a batch of 1,048,576
independent Ed25519 signatures over 32-byte block digests (seed_i =
SHA-512("mysti-seed"||i)[:32], msg_i = Blake2b-256("mysti-msg"||i), RFC 8032
signatures made on the GPU by the library's own signer), verified with ZIP-215
semantics. One step = one verify pass over the whole batch, inputs and the accept
vector resident in HBM (no PCIe in the timed region; the PCIe-inclusive rate is
reported separately as `end_to_end`).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--cpu-sample S]

N > 1: one rank per GPU under torch.distributed.run. Launched bare (`bench.py --gpus N`,
no WORLD_SIZE), the script starts that launcher itself as a child process before any
GPU call and exits with its code; under an external launcher WORLD_SIZE must equal N.
Each rank verifies its own shard (weak scaling, no data-path collective); barrier +
synchronize around the timed region, max time over ranks (gloo), value = all ranks'
signatures / that time.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import math
import os
import struct
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "verified StatementBlock sigs/sec (1/2/4/8 MI355X) vs host-core ed25519-consensus"
# Work accounting. Unit: one field multiplication or squaring = 64
# 32x32->64 multiply-accumulates (SURVEY.md §8d convention), each MAC 2 full-rate issue
# slots; hashes in 32-bit ops (SHA-512 compression ~6,000, BLAKE2b compression 2,688).
#   reference algorithm (dalek single verify, §8d): 3,200 field ops + 1 SHA-512
#   k_bv_prep (batch path): ZIP-215 decode of A and R = 2 x (255 sq + 23 mul), the
#       precomp conversion included, + SHA-512 (k) + BLAKE2b (z)
#   whole batch step: prep + 24 bucket additions x 7 field ops (+ ~2 for the tree)
#   k_verify (single path): decode 2 x 278 + tables 126 + 32-window ladder 1,632 + 21
FIELD_MACS = 64
W_SHA512_OPS = 6000
W_BLAKE2B_OPS = 2688
F_REFERENCE = 3200
F_PREP = 2 * (255 + 23)
F_BATCH_STEP = F_PREP + 24 * 7 + 2
F_SINGLE = 2 * 278 + 126 + 1632 + 21
# Peaks: full-rate 32-bit VALU = 256 CU x 128 lanes/clk x 2.4 GHz (MI355X_MICROARCH.md:
# FP32 vector 157.3 TFLOPS = 2 x 78.6 T lane-ops/s); v_mad_u64_u32 issues at half that
# rate on gfx950 (tools/microbench_valu.hip, profiles/r01_microbench_valu*.jsonl), so one
# MAC costs 2 full-rate issue slots.
PEAK_VALU_OPS = 256 * 128 * 2.4e9
MAC_SLOTS = 2
PEAK_MAC = PEAK_VALU_OPS / MAC_SLOTS  # v_mad_u64_u32 (half rate): 3.93e13 MACs/s
# SURVEY.md 8(d)'s fixed per-signature work: W_verify = 3,200 field ops x 64 MACs at the MAC
# peak, W_sha512 = 6,000 ops at the full-rate peak (the dalek single-verify algorithm)
W8D_SECONDS_PER_SIG = F_REFERENCE * FIELD_MACS / PEAK_MAC + W_SHA512_OPS / PEAK_VALU_OPS


def slots(field_ops: int, hash_ops: int) -> int:
    """Full-rate VALU issue slots for `field_ops` field multiplications plus hash ops."""
    return field_ops * FIELD_MACS * MAC_SLOTS + hash_ops


def pmc_traffic(kernel: str, workload: str = "c2"):
    """HBM bytes per launch of `kernel` from the newest committed PMC summary (profiles/<round>/
    pmc_<workload>_<kernel>.json from tools/gpu.sh pmc:W, or the round-1 pmc_<kernel>.json)."""
    import glob

    files = []
    # (pmc_<W>s1_: the pass ran the workload on one stream, as tools/gpu.sh pmc:c2s1 / pmc:c4s1 do)
    for pat in (f"pmc_{workload}_{kernel}.json", f"pmc_{workload}s1_{kernel}.json", f"pmc_{kernel}.json"):
        files += glob.glob(os.path.join(ROOT, "profiles", "**", pat), recursive=True)
    rnd = lambda p: os.path.relpath(p, os.path.join(ROOT, "profiles")).split(os.sep)[0]  # r01, r02, ...
    mine = lambda p: os.path.basename(p).startswith((f"pmc_{workload}_", f"pmc_{workload}s1_"))
    for f in sorted(files, key=lambda p: (rnd(p), "final" in p, mine(p)), reverse=True):
        try:
            d = json.load(open(f))
            return d.get("hbm_bytes_per_launch"), os.path.relpath(f, ROOT)
        except (OSError, ValueError):
            continue
    return None, None


def corpus_host(lo: int, n: int):
    seed = np.frombuffer(b"".join(hashlib.sha512(b"mysti-seed" + struct.pack("<Q", i)).digest()[:32]
                                  for i in range(lo, lo + n)), dtype=np.uint8).reshape(n, 32)
    msg = np.frombuffer(b"".join(hashlib.blake2b(b"mysti-msg" + struct.pack("<Q", i), digest_size=32).digest()
                                 for i in range(lo, lo + n)), dtype=np.uint8).reshape(n, 32)
    return seed, msg


def openssl_baseline(pk: np.ndarray, sig: np.ndarray, msg: np.ndarray, n: int, threads: int):
    """BASELINE.md 2's secondary CPU speed reference: OpenSSL libcrypto Ed25519 EVP_DigestVerify
    (bench_native/openssl_ed25519.c, built here against the system libcrypto) on the first n
    config-2 signatures, one core and `threads` cores. Strict RFC 8032 semantics, not ZIP-215:
    a speed reference on valid signatures only. None when libcrypto or its headers are absent."""
    import ctypes

    src = os.path.join(ROOT, "bench_native", "openssl_ed25519.c")
    so = os.path.join(ROOT, "bench_native", "build", "libmv_openssl.so")
    try:
        if not os.path.exists(so) or os.path.getmtime(so) < os.path.getmtime(src):
            os.makedirs(os.path.dirname(so), exist_ok=True)
            subprocess.run(["gcc", "-O2", "-fPIC", "-shared", "-pthread", "-o", so, src, "-lcrypto"], check=True,
                           stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        lib = ctypes.CDLL(so)
    except (OSError, subprocess.CalledProcessError):
        return None
    vp = ctypes.c_void_p
    lib.mvb_openssl_verify.argtypes = [vp, vp, vp, ctypes.c_size_t, vp, ctypes.c_int]
    lib.mvb_openssl_verify.restype = ctypes.c_int
    res = {}
    for t, m in ((1, min(n, 1 << 16)), (threads, n)):
        p = np.ascontiguousarray(pk[:m]); s = np.ascontiguousarray(sig[:m]); g = np.ascontiguousarray(msg[:m])
        st = np.ones(m, dtype=np.uint8)
        t0 = time.perf_counter()
        rc = lib.mvb_openssl_verify(vp(p.ctypes.data), vp(s.ctypes.data), vp(g.ctypes.data), m, vp(st.ctypes.data), t)
        dt = time.perf_counter() - t0
        if rc != 0:
            return None
        res[t] = (m / dt, m, dt, int((st == 0).sum()))
    return {"value": round(res[threads][0], 1), "unit": "sigs/s", "cores": threads,
            "single_core_value": round(res[1][0], 1),
            "accepted": res[threads][3], "of": res[threads][1],
            "sample": f"{res[threads][1]} config-2 signatures on {threads} threads ({res[threads][2]:.1f} s); "
                      f"single core: {res[1][1]} ({res[1][2]:.1f} s)",
            "note": "OpenSSL libcrypto Ed25519 EVP_DigestVerify (BASELINE.md 2 secondary reference): strict "
                    "RFC 8032, cofactorless -- a speed reference on valid signatures, not the reference's "
                    "ZIP-215 semantics; the key is decoded per signature (distinct keys)"}


def cpu_baseline(pk: np.ndarray, sig: np.ndarray, msg: np.ndarray, sample: int):
    """The oracle's C restatement (-O3 -march=native, built on this host) on a bounded sample."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "-s", "native"], check=True)
    import ctypes

    from mysticeti_amd.dist import cpu_share

    lib = ctypes.CDLL(os.path.join(ROOT, "oracle", "build", "libmv_oracle_native.so"))
    vp = ctypes.c_void_p
    lib.orc_ed25519_verify_batch.argtypes = [vp, vp, vp, ctypes.c_size_t, vp, ctypes.c_int]
    threads, share_src = cpu_share()
    res = {}
    # ~8 s single-threaded, then `passes` sweeps of the sample on all threads (~10 s)
    for t, n, passes in ((1, min(sample, 250_000), 1), (threads, sample, 4)):
        p = np.ascontiguousarray(pk[:n]); s = np.ascontiguousarray(sig[:n]); m = np.ascontiguousarray(msg[:n])
        st = np.zeros(n, dtype=np.uint8)
        t0 = time.perf_counter()
        for _ in range(passes):
            lib.orc_ed25519_verify_batch(vp(p.ctypes.data), vp(s.ctypes.data), vp(m.ctypes.data), n,
                                         vp(st.ctypes.data), t)
        dt = time.perf_counter() - t0
        assert (st == 0).all(), "oracle rejected a valid corpus signature"
        res[t] = (n * passes / dt, n * passes, dt)
    ossl = openssl_baseline(pk, sig, msg, min(sample, 1 << 18), threads)
    model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {
        "value": round(res[threads][0], 1), "unit": "sigs/s", "cores": threads, "kind": "port",
        "sample": f"{res[threads][1]} verifies of config-2 signatures on {threads} threads ({res[threads][2]:.1f} s); "
                  f"single core: {res[1][1]} verifies ({res[1][2]:.1f} s)",
        "single_core_value": round(res[1][0], 1), "host_cpu": model, "nproc": os.cpu_count(),
        "cores_source": share_src, "openssl": ossl,
        "impl": "oracle/ed25519.c: dalek u64-backend structure (5x51 limbs, Straus wNAF-5/8), gcc -O3 -march=native",
    }


# Keys dropped below the top level of the stdout line (compact_line): prose and per-leg detail.
# The driver keeps only the last ~8 KB of stdout; the full line goes to stderr.
_VERBOSE = {"note", "impl", "host_cpu", "nproc", "data", "label", "kernel_ms_source", "frac_label", "work_per_sig",
            "work", "per", "traffic_source", "stage_ms_as_run", "sha256_msg_digests_first_corpus", "mean_us",
            "batches", "unit", "cpu_1t", "rss_after", "hbm_peak_at", "queue_calls", "online_launches",
            "online_requests", "values", "bincode_GB", "seconds", "host_enqueue", "sample", "cores_source", "config",
            "traffic_per_2^20_blocks", "work_per_block", "entries_per_s", "hbm_bincode_GBps"}


def _prune(x, depth=0):
    if isinstance(x, dict):
        return {k: _prune(v, depth + 1) for k, v in x.items() if not (depth > 0 and k in _VERBOSE)}
    if isinstance(x, list):
        return [_prune(v, depth + 1) for v in x]
    if isinstance(x, float):
        return float(f"{x:.5g}") if abs(x) < 1e5 else round(x, 1)
    return x


def summary_of(out: dict) -> dict:
    """Every leg's headline in one flat dict (the last key of the stdout line, so it survives any
    tail of the driver's record). Units: sigs/s, blocks/s, GB/s, ms, us."""
    g = lambda d, *ks: None if d is None else (d.get(ks[0]) if len(ks) == 1 else g(d.get(ks[0]), *ks[1:]))
    s = {"c2_sigs_per_s": out["value"], "c2_ms_per_step": out["ms_per_step"],
         "c2_sustained_median": g(out, "sustained", "median"), "c2_prep_frac": g(out, "roofline", "frac"),
         "c2_step_frac": g(out, "pipeline", "frac"),
         "c3_1pct_sigs_per_s": g(out, "adversarial", "config3_1pct", "value"),
         "one_bad_per_batch_sigs_per_s": g(out, "adversarial", "one_bad_per_batch", "value"),
         "e2e_pinned_sigs_per_s": g(out, "end_to_end", "value"),
         "e2e_frac_of_resident": round(out["end_to_end"]["value"] / out["value"], 4) if out.get("end_to_end") else None,
         "e2e_two_callers_sigs_per_s": g(out, "end_to_end", "two_callers", "value"),
         "c4_blocks_per_s": g(out, "config4", "value"), "c4_ms_per_step": g(out, "config4", "ms_per_step"),
         "c4_kernel_frac": g(out, "config4", "roofline", "frac"),
         "c4_traffic_over_bincode": g(out, "config4", "roofline", "traffic_over_bincode"),
         "c4_host_fed_blocks_per_s": g(out, "config4", "host_fed", "value"),
         "wal_GBps": g(out, "wal", "value"), "cpu_sigs_per_s": g(out, "cpu_baseline", "value"),
         "cpu_cores": g(out, "cpu_baseline", "cores"),
         "cpu_openssl_sigs_per_s": g(out, "cpu_baseline", "openssl", "value")}
    shapes = g(out, "config5", "shapes") or {}
    for k, v in shapes.items():
        s[f"c5_{k}_64blk_p50_us"] = g(v, "gpu", "p50_us")
        s[f"c5_{k}_64blk_cpu_p50_us"] = g(v, "cpu_16t", "p50_us")
        for leg in ("concurrent_1_block_callers", "fan_in_callers"):
            c = v.get(leg)
            if c:
                s[f"c5_{k}_{c['callers']}callers_gpu_over_cpu"] = c.get("gpu_over_cpu_blocks_per_s")
    s["correct"] = out["correct"]
    s["parity_sha256"] = out.get("parity_sha256")
    return {k: v for k, v in s.items() if v is not None}


def compact_line(out: dict) -> dict:
    c = _prune(out)
    c["summary"] = summary_of(out)
    return c


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # default timed region >= 2 s (600 steps of ~3.5 ms; BASELINE.md 2: DVFS settles)
    ap.add_argument("--steps", type=int, default=600)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch", type=int, default=1 << 20, help="signatures per GPU per step")
    ap.add_argument("--cpu-sample", type=int, default=1 << 20, help="0 disables the CPU baseline")
    ap.add_argument("--no-e2e", action="store_true")
    ap.add_argument("--streams", type=int, default=3, help="batch path: streams the steps rotate over (3: profiles/r05/c2_streams_slots.txt)")
    ap.add_argument("--path", choices=["batch", "single"], default="batch",
                    help="batch: one combined equation per step (batch.hip) with exact fallback; "
                         "single: every signature verified alone (k_verify)")
    ap.add_argument("--workload", choices=["config2", "config4", "config5", "wal"], default="config2",
                    help="config2 (default, the headline line): 1M independent signatures per GPU; "
                         "config4: HBM-resident 100-validator blocks through the device block pipeline; "
                         "config5: p50/p99 latency of 64-block batches, GPU vs host cores; "
                         "wal: WAL replay check (SURVEY.md 8 f4) over an HBM-resident image")
    ap.add_argument("--batches", type=int, default=10000, help="config5: GPU batches timed per shape")
    ap.add_argument("--conc-seconds", type=float, default=3.0, help="config5: seconds of concurrent 1-block callers")
    ap.add_argument("--corrupt", type=int, default=0, help="signatures per batch with a flipped s bit")
    ap.add_argument("--groups", type=int, default=0, help="sub-batch equations per batch (0 = adaptive)")
    ap.add_argument("--sustain-repeats", type=int, default=5, help="repeats of the sustained-rate measurement")
    ap.add_argument("--sustain-seconds", type=float, default=2.0, help="seconds per sustained repeat")
    ap.add_argument("--no-adversarial", dest="adversarial", action="store_false",
                    help="skip the 1-bad-signature and config-3 (1%% corrupted) rates")
    ap.add_argument("--no-config4", dest="config4", action="store_false",
                    help="skip the config-4 (100-validator blocks) rate in the default line")
    ap.add_argument("--config4-batch", type=int, default=1 << 21,
                    help="config-4 blocks per GPU per step (2^21: BASELINE config 4's 16M blocks over 8 GPUs)")
    ap.add_argument("--host-fed-blocks", type=int, default=1 << 17,
                    help="config 4's PCIe-inclusive leg: blocks fed from host memory (0 disables)")
    ap.add_argument("--no-config5", dest="config5", action="store_false",
                    help="skip the config-5 (online latency) key of the default line")
    ap.add_argument("--config5-batches", type=int, default=2000,
                    help="default line's config-5 leg: 64-block calls timed per shape")
    ap.add_argument("--config5-seconds", type=float, default=2.0,
                    help="default line's config-5 leg: seconds of concurrent 1-block callers per shape")
    ap.add_argument("--conc-callers", type=int, default=0,
                    help="config 5: the concurrent-callers leg's callers (0: the CPU share's thread count)")
    ap.add_argument("--fanin-callers", type=int, default=99,
                    help="config 5: the fan-in leg's concurrent 1-block callers (committee - 1 of config 4's "
                         "100-validator committee; 0 disables)")
    ap.add_argument("--no-wal", dest="wal", action="store_false",
                    help="skip the WAL replay-check rate (row f4) in the default line")
    ap.add_argument("--wal-entries", type=int, default=1 << 20, help="WAL entries (config-4 blocks) per GPU")
    args = ap.parse_args()
    from mysticeti_amd.dist import launch_ranks, needs_launch

    if needs_launch(args.gpus):
        # `bench.py --gpus N` without an external launcher: start the N ranks as a child
        # torch.distributed.run (nothing here has touched the GPU) and exit with its code
        return launch_ranks(os.path.abspath(__file__), sys.argv[1:], args.gpus)
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    if world_env != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world_env}")
    if args.workload != "config2":
        import bench_blocks

        return bench_blocks.run(args)

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    # the CPU baselines run on rank 0 of a one-GPU run only: the N > 1 lines of a scaling run
    # report the GPUs alone (and finish sooner); config 5's GPU-vs-CPU latency leg keeps its CPU side
    cpu_legs = args.cpu_sample > 0 and world == 1
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
    dev = torch.device("cuda", local_rank)
    import mysticeti_amd as M
    from mysticeti_amd.dist import all_ranks_ok, footprint, hbm_sample, rss_mark, shard_range, timed_region

    def progress(what):  # one stderr line per leg (a long run shows it is alive)
        if rank == 0:
            print(f"bench: {what} ({time.strftime('%H:%M:%S')})", file=sys.stderr, flush=True)

    eng = M.Engine(devices=(local_rank,))
    if "MV_PREP_CHAIN" not in os.environ:
        # the steps rotate over this script's own streams: let each step's k_bv_prep follow the
        # previous one's on them too (the library chains only its own streams by default)
        eng.set_option("MV_PREP_CHAIN", 2)
    n = args.batch

    # ---- corpus: host hashes, GPU signing (library signer), all resident in HBM ----
    lo, _ = shard_range(rank, world, n)
    seed_h, msg_h = corpus_host(lo, n)
    d_seed = torch.from_numpy(seed_h.copy()).to(dev)
    d_msg = torch.from_numpy(msg_h.copy()).to(dev)
    d_pk = torch.empty((n, 32), dtype=torch.uint8, device=dev)
    d_sig = torch.empty((n, 64), dtype=torch.uint8, device=dev)
    # dedicated non-default streams: the library launches on them and the HIP events
    # below are recorded on them, so kernel_ms times exactly the verify launches. The
    # batch path rotates over three streams so that one batch's latency-bound tail (window
    # reduction, final check: a few waves) runs beside the next batches' full-chip kernels
    # (three streams and three engine scratch slots: 316-319 M/s against 295-299 M/s on two,
    # profiles/r05/c2_streams_slots.txt).
    nstreams = args.streams if args.path == "batch" else 1
    streams = [torch.cuda.Stream(dev) for _ in range(nstreams)]
    assert all(st.cuda_stream != 0 for st in streams)
    d_status = [torch.full((n,), 255, dtype=torch.uint8, device=dev) for _ in range(nstreams)]
    d_ok = [torch.zeros(1, dtype=torch.int32, device=dev) for _ in range(nstreams)]
    torch.cuda.synchronize(dev)  # the H2D copies above ran on the default stream
    eng.dev_sign(local_rank, d_seed, d_msg, d_pk, d_sig, streams[0].cuda_stream)
    torch.cuda.synchronize(dev)
    bad_idx = None
    if args.corrupt:
        bad_idx = torch.linspace(0, n - 1, args.corrupt, device=dev).long() if args.corrupt > 1 else \
            torch.tensor([n // 3], device=dev)
        d_sig[bad_idx, 40] ^= 0x10  # s bit: s stays < l, R decodes -> only the equation catches it
    if args.groups:
        eng.set_batch_groups(args.groups)

    state = {"i": 0}

    def step():
        j = state["i"] % nstreams
        state["i"] += 1
        if args.path == "batch":
            eng.dev_verify_batch(local_rank, d_msg, d_sig, d_pk, d_status[j], d_ok[j], streams[j].cuda_stream)
        else:
            eng.dev_verify(local_rank, d_msg, d_sig, d_pk, d_status[j], streams[j].cuda_stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    hbm_sample(torch, dev, "config2")
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev_side = [torch.cuda.Event() for _ in range(nstreams)]

    def timed_step():
        if state["i"] == args.warmup:
            ev0.record(streams[0])  # HIP events on the launch streams bracket the K steps
            for st in streams[1:]:
                st.wait_event(ev0)
        step()

    def close_and_sync():
        if state["i"] > args.warmup:
            for st, ev in zip(streams[1:], ev_side[1:]):
                ev.record(st)
                streams[0].wait_event(ev)
            ev1.record(streams[0])
        torch.cuda.synchronize(dev)

    progress("corpus ready, timed region")
    elapsed = timed_region(timed_step, args.steps, close_and_sync, dist)
    kernel_ms = ev0.elapsed_time(ev1) / args.steps  # device time per step on the launch streams
    stage_ms = {}
    if args.path == "batch":
        # the as-run stage table: HIP events around every stage of a few more steps on the same
        # alternating streams, after the timed region (the events stay out of `value`)
        eng.stage_times(reset=True)
        eng.set_stage_timing(True)
        for _ in range(max(2 * nstreams, min(args.steps, 20))):
            step()
        torch.cuda.synchronize(dev)
        tot, calls = eng.stage_times()
        eng.set_stage_timing(False)
        stage_ms = {k: v / calls[k] for k, v in tot.items() if calls[k]}
    # With two streams a stage's events also count time its kernels share the chip with the
    # other stream's tail. Re-time the stages on ONE stream after the timed region (untimed
    # for `value`), so the dominant kernel's duration matches the single-stream rocprof trace
    # (profiles/<round>/, tools/gpu.sh trace:c2s1).
    iso_ms = {}
    if args.path == "batch" and nstreams > 1:
        eng.stage_times(reset=True)
        eng.set_stage_timing(True)
        for _ in range(3):
            eng.dev_verify_batch(local_rank, d_msg, d_sig, d_pk, d_status[0], d_ok[0], streams[0].cuda_stream)
        torch.cuda.synchronize(dev)
        tot, calls = eng.stage_times()
        eng.set_stage_timing(False)
        iso_ms = {k: v / calls[k] for k, v in tot.items() if calls[k]}
    batch_ok = all(int(x.item()) == 1 for x in d_ok) if args.path == "batch" else None

    status = d_status[(args.warmup + args.steps - 1) % nstreams].cpu().numpy()
    accepted = int((status == 0).sum())
    if bad_idx is None:
        ok = accepted == n and all((x.cpu().numpy() == 0).all() for x in d_status)
    else:
        want = np.zeros(n, np.uint8)
        want[bad_idx.cpu().numpy()] = 1
        ok = all((x.cpu().numpy() == want).all() for x in d_status)
    parity = None
    if rank == 0 and n == (1 << 20) and bad_idx is None:
        gold = json.load(open(os.path.join(ROOT, "tests", "golden", "batch_config2.json")))
        parity = hashlib.sha256(status.tobytes()).hexdigest() == gold["sha256_status"] and \
            hashlib.sha256(d_sig.cpu().numpy().tobytes()).hexdigest() == gold["sha256_sig"]
    ok = all_ranks_ok(ok, dist)

    total = n * world * args.steps
    value = total / elapsed
    if args.path == "batch":
        # headline roofline: k_bv_prep's real work over its single-stream time (the stage
        # events of the post-run one-stream steps; the 2-stream as-run time is reported beside)
        kern, kern_ms = "k_bv_prep", iso_ms.get("prep", stage_ms["prep"])
        w_kern = slots(F_PREP, W_SHA512_OPS + W_BLAKE2B_OPS)
        w_step = slots(F_BATCH_STEP, W_SHA512_OPS + W_BLAKE2B_OPS)
        kdesc = (f"{F_PREP} field ops x {FIELD_MACS} MACs x {MAC_SLOTS} slots + SHA-512 {W_SHA512_OPS} + "
                 f"BLAKE2b {W_BLAKE2B_OPS} ops per signature")
    else:
        kern, kern_ms = "k_verify", kernel_ms
        w_kern = w_step = slots(F_SINGLE, W_SHA512_OPS)
        kdesc = f"{F_SINGLE} field ops x {FIELD_MACS} MACs x {MAC_SLOTS} slots + SHA-512 {W_SHA512_OPS} ops"
    achieved = n / (kern_ms * 1e-3) * w_kern
    traffic, traffic_src = pmc_traffic(kern)

    # sustained rate: >= 5 repeats of >= 2 s each (DVFS settles), median
    sustained = None
    if args.sustain_repeats > 0:
        per = max(args.steps, int(math.ceil(args.sustain_seconds / max(elapsed / args.steps, 1e-4))))
        vals = []
        for _ in range(args.sustain_repeats):
            e = timed_region(step, per, lambda: torch.cuda.synchronize(dev), dist)
            vals.append(n * world * per / e)
        sustained = {"repeats": len(vals), "steps_each": per, "seconds_each": round(per * elapsed / args.steps, 2),
                     "values": [round(v, 1) for v in vals], "median": round(float(np.median(vals)), 1),
                     "frac_of_value": round(float(np.median(vals)) / value, 4)}

    # adversarial batches (config 3 / a Byzantine signer): corrupted copies of the corpus,
    # verdicts checked against the expected mask; each rate after 9 untimed steps (the
    # adaptive policy's steady state: a failed equation cuts the next batches into groups, and
    # dense failures send them to the single path; with three streams in flight the policy
    # sees a batch's flags about three batches later)
    adversarial = None
    if args.path == "batch" and args.adversarial and not args.corrupt:
        adversarial = {}
        rng = np.random.default_rng(2025)
        for name, idx in (("one_bad_per_batch", np.array([n // 3])),
                          ("config3_1pct", np.sort(rng.choice(n, n // 100, replace=False)))):
            d_bad = d_sig.clone()
            t_idx = torch.from_numpy(idx).to(dev)
            d_bad[t_idx, 40] ^= 0x10  # s bit: s stays < l and R decodes: only an equation catches it
            want = np.zeros(n, np.uint8)
            want[idx] = 1
            st = {"i": 0}

            def adv_step():
                j = st["i"] % nstreams
                st["i"] += 1
                eng.dev_verify_batch(local_rank, d_msg, d_bad, d_pk, d_status[j], d_ok[j], streams[j].cuda_stream)

            for _ in range(9):
                adv_step()
            torch.cuda.synchronize(dev)
            c0, r0 = eng.batch_counters(), eng.batch_routes()
            k = max(4, min(args.steps // 2, 200))
            e = timed_region(adv_step, k, lambda: torch.cuda.synchronize(dev), dist)
            c1, r1 = eng.batch_counters(), eng.batch_routes()
            good = all((x.cpu().numpy() == want).all() for x in d_status)
            ok = ok and good
            rate = n * world * k / e
            adversarial[name] = {"value": round(rate, 1), "unit": "sigs/s", "steps": k,
                                 "bad_signatures_per_batch": int(idx.size),
                                 "ratio_to_all_valid": round(rate / value, 4), "correct": bool(good),
                                 "groups_per_batch": round((c1[2] - c0[2]) / max(1, c1[0] - c0[0]), 2),
                                 "groups_reverified_per_batch": round((c1[3] - c0[3]) / max(1, c1[0] - c0[0]), 2),
                                 "single_path_batches": r1[1] - r0[1], "equation_batches": r1[0] - r0[0]}
            del d_bad
        adversarial["note"] = ("one flipped s bit per bad signature (s < l, R decodes); the batch is re-verified "
                               "only in the sub-batch equations that fail; dense failures go straight to the "
                               "single path (DESIGN.md 2)")
        ok = all_ranks_ok(ok, dist)
        # the adversarial batches armed the guard (the next 64 batches in 8 sub-batch equations):
        # the legs below measure the unguarded default
        eng.set_batch_groups(args.groups)

    rss_mark("adversarial")
    progress("adversarial done")
    # PCIe-inclusive rates (host buffers through the C ABI)
    e2e = None
    if rank == 0 and not args.no_e2e:
        # PCIe-inclusive: host buffers in, accept vector out, through the C ABI
        pk_h, sig_h = d_pk.cpu().numpy(), d_sig.cpu().numpy()

        def e2e_rate(m_, s_, p_, reps=3):
            eng.ed25519_verify(m_, s_, p_)
            best, st_ = None, None
            for _ in range(reps):
                t2 = time.perf_counter()
                st_ = eng.ed25519_verify(m_, s_, p_)
                dt = time.perf_counter() - t2
                best = dt if best is None else min(best, dt)
            return n / best, int((st_ == 0).sum())

        v_page, acc_page = e2e_rate(msg_h, sig_h, pk_h)
        # the same arrays in page-locked memory (mv_host_alloc): chunked H2D beside the verify
        pm, ps, pp = eng.host_empty(msg_h.shape), eng.host_empty(sig_h.shape), eng.host_empty(pk_h.shape)
        pm[:], ps[:], pp[:] = msg_h, sig_h, pk_h
        v_pin, acc_pin = e2e_rate(pm, ps, pp)
        # two callers at once (the reference verifies in one task per peer, net_sync.rs:214-221):
        # each its own pinned copy of the corpus; aggregate = both calls' signatures / wall time
        import threading

        pm2, ps2, pp2 = eng.host_empty(msg_h.shape), eng.host_empty(sig_h.shape), eng.host_empty(pk_h.shape)
        pm2[:], ps2[:], pp2[:] = msg_h, sig_h, pk_h
        two_ok = []

        def two_callers():
            outs = [None, None]

            def call(c, a):
                outs[c] = eng.ed25519_verify(*a)

            th = [threading.Thread(target=call, args=(c, a)) for c, a in enumerate(((pm, ps, pp), (pm2, ps2, pp2)))]
            t2 = time.perf_counter()
            for x in th:
                x.start()
            for x in th:
                x.join()
            dt = time.perf_counter() - t2
            two_ok.append(all(o is not None and int((o == 0).sum()) == n for o in outs))
            return dt

        two_callers()
        v_two = 2 * n / min(two_callers() for _ in range(3))
        e2e = {"value": round(v_pin, 1), "unit": "sigs/s",
               "two_callers": {"value": round(v_two, 1), "frac_of_resident": round(v_two / value, 4),
                               "correct": all(two_ok),
                               "note": "two threads, each mv_ed25519_verify on its own pinned copy of the "
                                       "corpus at once; aggregate signatures / wall time, best of 3"},
               "note": "host arrays in, statuses out (H2D 128 B/sig), best of 3 calls; value: inputs in pinned "
                       "memory (mv_host_alloc), chunked copies beside the verify; pageable: plain numpy arrays",
               "pageable": round(v_page, 1), "accepted": acc_pin, "accepted_pageable": acc_page}
        ok = ok and all(two_ok)
        del pm2, ps2, pp2

    rss_mark("end_to_end")
    progress("end_to_end done")
    # config 4 (the largest workload): whole-block verification of HBM-resident 100-validator
    # blocks, measured in the same run (bench_blocks.config4_measure)
    cfg4 = None
    if args.config4 and args.path == "batch" and not args.corrupt:
        import bench_blocks

        cfg4 = bench_blocks.config4_measure(eng, torch, local_rank, world, dist, n=args.config4_batch,
                                            steps=max(3, min(args.steps, 100)), warmup=max(4, min(args.warmup, 8)),
                                            nstreams=nstreams,
                                            cpu=cpu_legs, host_blocks=args.host_fed_blocks)
        ok = ok and cfg4["correct"]

    rss_mark("config4")
    progress("config4 done")
    # f4: the WAL replay check over an HBM-resident WAL of config-4 blocks (bench_wal.wal_measure)
    walr = None
    if args.wal and args.path == "batch" and not args.corrupt:
        import bench_wal

        walr = bench_wal.wal_measure(eng, torch, local_rank, world, dist, n=args.wal_entries,
                                     steps=max(3, min(args.steps // 4, 50)), warmup=1, cpu=cpu_legs)
        ok = ok and walr["correct"]

    rss_mark("wal")
    progress("wal done")
    # config 5 (the online path): latency of 64-block calls and concurrent 1-block callers through
    # mv_verify_blocks on host buffers, GPU and CPU in the same run (bench_blocks.config5_measure);
    # rank 0 only (the host CPU legs would otherwise compete across ranks)
    cfg5 = None
    if args.config5 and args.path == "batch" and not args.corrupt and rank == 0:
        import bench_blocks

        eng.set_batch_groups(args.groups)
        cfg5 = bench_blocks.config5_measure(eng, batches=args.config5_batches, conc_seconds=args.config5_seconds,
                                            cpu=args.cpu_sample > 0, fanin_callers=args.fanin_callers,
                                            callers=args.conc_callers or None)
        ok = ok and cfg5["correct"]

    rss_mark("config5")
    progress("config5 done")
    cpu = None
    if rank == 0 and cpu_legs:
        cpu = cpu_baseline(d_pk.cpu().numpy(), d_sig.cpu().numpy(), msg_h, min(args.cpu_sample, n))
        rss_mark("cpu_baseline")
    # per-rank peak host RSS and HBM in use (all ranks; the line must hold at 8 ranks per node)
    fp = footprint(rank, dist)
    out = None
    if rank == 0:
        out = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "sigs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (config-2 corpus regenerated from its seed rule; signed on-GPU, pinned by "
                    "tests/golden/batch_config2.json)",
            "config": {"workload": "config2: 1,048,576 independent Ed25519 (ZIP-215) signatures over 32-byte "
                                   "block digests per GPU", "batch_per_gpu": n, "global_batch": n * world,
                       "parallelism": f"shard-per-gpu x{world}, no collective"},
            "roofline": {"bound": "valu", "achieved": round(achieved / 1e12, 3), "peak": round(PEAK_VALU_OPS / 1e12, 2),
                         "unit": "TOP/s", "frac": round(achieved / PEAK_VALU_OPS, 4), "traffic": traffic,
                         "traffic_source": traffic_src, "kernel": kern, "kernel_ms": round(kern_ms, 4),
                         "kernel_ms_source": "HIP events on the launch stream around k_bv_prep, 3 post-run steps "
                                             "on ONE stream (compare profiles/<round>/kernel_stats_config2_1stream.csv)",
                         "kernel_ms_as_run": round(stage_ms.get("prep", kern_ms), 4) if stage_ms else None,
                         "frac_label": "real work of the dominant kernel: its field ops and hashes at the full-rate "
                                       "INT32 VALU peak",
                         "work_per_sig": kdesc,
                         "frac_8d": {"value": round(value / world * W8D_SECONDS_PER_SIG, 4),
                                     "label": "SURVEY.md 8(d) fixed work (W_verify = 3,200 field ops x 64 MACs at the "
                                              "v_mad_u64_u32 peak 39.3 T/s + W_sha512 6,000 ops at 78.6 T/s) x "
                                              "value; exceeds 1 because the batch algorithm does ~726 field ops "
                                              "per signature, not the single-verify 3,200"},
                         "stage_ms_one_stream": {k: round(v, 4) for k, v in iso_ms.items()} if iso_ms else None},
            "pipeline": {"device_ms_per_step": round(kernel_ms, 4),
                         "stage_ms": {k: round(v, 4) for k, v in stage_ms.items()} if stage_ms else None,
                         "achieved_TOPs": round(value / world * w_step / 1e12, 3),
                         "frac": round(value / world * w_step / PEAK_VALU_OPS, 4),
                         "work_per_sig_field_ops": F_BATCH_STEP if args.path == "batch" else F_SINGLE,
                         "reference_equivalent_TOPs": round(value / world * slots(F_REFERENCE, W_SHA512_OPS) / 1e12, 3),
                         "note": "reference_equivalent counts the dalek single-verify work (3,200 field ops, "
                                 "SURVEY.md 8d) per verified signature; it is not a roofline fraction"},
            "cpu_baseline": cpu,
            "sustained": sustained,
            "adversarial": adversarial,
            "config4": cfg4,
            "config5": cfg5,
            "wal": walr,
            "end_to_end": e2e,
            "footprint": {"per_rank": fp, "note": "host_rss_peak_GB: getrusage ru_maxrss (pinned staging included); "
                                                  "hbm_peak_GB: largest hipMemGetInfo total - free seen after each "
                                                  "leg's warm-up (device-wide)"},
            "correct": bool(ok),
            "path": args.path,
            "batch_equation_held": batch_ok,
            "parity_sha256": parity,
        }
        if cpu:
            out["speedup_vs_cpu"] = {"all_cores": round(value / world / cpu["value"], 1),
                                     "single_core": round(value / world / cpu["single_core_value"], 1)}
        # the full line on stderr, the compact one (every leg's headline in `summary`, its last
        # key) on stdout: the driver's record keeps the stdout tail
        print("bench_full_line: " + json.dumps(out), file=sys.stderr, flush=True)
        print(json.dumps(compact_line(out)), flush=True)
    eng.close()
    if dist:
        dist.destroy_process_group()
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
