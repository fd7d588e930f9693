"""Diagnostics: host-buffer verify timing, pageable arrays vs pinned ones (mv_host_alloc; the
streamed path: chunked DMA copies gate k_bv_prep). MV_STREAM_CHUNK_LOG2 sets its chunk size."""
import os, sys, time
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
torch.cuda.init()
import mysticeti_amd as M
eng = M.Engine()
n = 1 << 20
rng = np.random.default_rng(1)
seed = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
msg = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
pk, sig = eng.ed25519_sign(seed, msg)


def rate(m, s, p, label):
    best = None
    for it in range(4):
        t0 = time.perf_counter(); st = eng.ed25519_verify(m, s, p); t1 = time.perf_counter()
        if it:
            best = t1 - t0 if best is None else min(best, t1 - t0)
    print(f"{label}: best {best * 1e3:.2f} ms -> {n / best / 1e6:.1f} M/s ok={bool((st == 0).all())}", flush=True)


rate(msg, sig, pk, "pageable")
pm, ps, pp = eng.host_empty(msg.shape), eng.host_empty(sig.shape), eng.host_empty(pk.shape)
pm[:], ps[:], pp[:] = msg, sig, pk
rate(pm, ps, pp, f"pinned chunk_log2={os.environ.get('MV_STREAM_CHUNK_LOG2', '17')}")
d = torch.empty(sig.shape, dtype=torch.uint8, device="cuda")
hp = torch.from_numpy(sig).pin_memory()
for _ in range(2):
    torch.cuda.synchronize()
    t0 = time.perf_counter(); d.copy_(hp, non_blocking=True); torch.cuda.synchronize(); t1 = time.perf_counter()
print(f"torch pinned H2D 64 MB: {(t1 - t0) * 1e3:.2f} ms = {sig.nbytes / (t1 - t0) / 1e9:.1f} GB/s", flush=True)
