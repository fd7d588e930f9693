"""Diagnostics: host-to-device copy rates from page-locked memory in the shapes the streamed
signature path uses (tools/gpu.sh h2d). 2^20 signatures = msg 32 MB + sig 64 MB + pk 32 MB,
copied (a) as three whole arrays on one stream, (b) in 2^17-signature chunks on one stream (the
engine's schedule: 24 copies), (c) the same chunks with the sig copies on a second stream, (d)
the chunks as one interleaved copy per chunk (one 128-B record per signature). Best of 5."""
import time

import torch

n = 1 << 20
chunk = 1 << 17
dev = torch.device("cuda", 0)
host = {k: torch.empty(n * w, dtype=torch.uint8).pin_memory() for k, w in (("msg", 32), ("sig", 64), ("pk", 32))}
rec = torch.empty(n * 128, dtype=torch.uint8).pin_memory()
devb = {k: torch.empty(v.numel(), dtype=torch.uint8, device=dev) for k, v in host.items()}
drec = torch.empty(rec.numel(), dtype=torch.uint8, device=dev)
s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
W = {"msg": 32, "sig": 64, "pk": 32}


def timed(fn):
    best = None
    for _ in range(6):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize(dev)
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
    return best


def whole():
    with torch.cuda.stream(s1):
        for k in host:
            devb[k].copy_(host[k], non_blocking=True)


def chunks(two):
    for o in range(0, n, chunk):
        for k in ("msg", "sig", "pk"):
            st = s2 if (two and k == "sig") else s1
            with torch.cuda.stream(st):
                w = W[k]
                devb[k][o * w:(o + chunk) * w].copy_(host[k][o * w:(o + chunk) * w], non_blocking=True)


def interleaved():
    with torch.cuda.stream(s1):
        for o in range(0, n, chunk):
            drec[o * 128:(o + chunk) * 128].copy_(rec[o * 128:(o + chunk) * 128], non_blocking=True)


mb = n * 128 / 1e6
for name, fn in (("three whole arrays, one stream", whole), ("2^17 chunks x 3 arrays, one stream", lambda: chunks(False)),
                 ("2^17 chunks, sig on a second stream", lambda: chunks(True)),
                 ("2^17 chunks of 128-B records, one stream", interleaved)):
    t = timed(fn)
    print(f"h2d {name}: {t * 1e3:.3f} ms, {mb / t / 1e3:.1f} GB/s", flush=True)
