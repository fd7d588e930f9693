"""Diagnostics: host-buffer verify timing (the pipelined path), per-chunk host stage times."""
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
for it in range(4):
    t0 = time.perf_counter(); st = eng.ed25519_verify(msg, sig, pk); t1 = time.perf_counter()
    print(f"call {it}: {(t1 - t0) * 1e3:.2f} ms -> {n / (t1 - t0) / 1e6:.1f} M/s ok={bool((st == 0).all())}", flush=True)
t0 = time.perf_counter(); a = np.empty_like(sig); a[:] = sig; t1 = time.perf_counter()
print(f"numpy memcpy 64 MB: {(t1 - t0) * 1e3:.2f} ms", flush=True)
d = torch.empty(sig.shape, dtype=torch.uint8, device="cuda")
torch.cuda.synchronize()
t0 = time.perf_counter(); d.copy_(torch.from_numpy(sig)); torch.cuda.synchronize(); t1 = time.perf_counter()
print(f"torch pageable H2D 64 MB: {(t1 - t0) * 1e3:.2f} ms", flush=True)
hp = torch.from_numpy(sig).pin_memory()
t0 = time.perf_counter(); d.copy_(hp, non_blocking=True); torch.cuda.synchronize(); t1 = time.perf_counter()
print(f"torch pinned H2D 64 MB: {(t1 - t0) * 1e3:.2f} ms", flush=True)
print("cpu_count", os.cpu_count(), "affinity", len(os.sched_getaffinity(0)))
