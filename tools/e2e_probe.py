"""Diagnostics: one pinned-input host verify of 2^20 signatures after two warm-up calls (the
streamed path), for a kernel + memory-copy timeline of the last call (tools/timeline.py)."""
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
pm, ps, pp = eng.host_empty(msg.shape), eng.host_empty(sig.shape), eng.host_empty(pk.shape)
pm[:], ps[:], pp[:] = msg, sig, pk
for it in range(3):
    time.sleep(0.05)
    t0 = time.perf_counter(); st = eng.ed25519_verify(pm, ps, pp); t1 = time.perf_counter()
    print(f"call {it}: {(t1 - t0) * 1e3:.2f} ms -> {n / (t1 - t0) / 1e6:.1f} M/s ok={bool((st == 0).all())}", flush=True)
