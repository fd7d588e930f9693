"""Diagnostics: pinned-input host verify of 2^20 signatures (the streamed path, mv_ed25519_verify
on mv_host_alloc arrays): best of 6 calls after two warm-ups, and the HBM-resident batch rate
of the same corpus beside it (tools/gpu.sh e2e:ENV=V,...)."""
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
best, ok = None, True
for it in range(8):
    t0 = time.perf_counter(); st = eng.ed25519_verify(pm, ps, pp); dt = time.perf_counter() - t0
    ok &= bool((st == 0).all())
    if it >= 2:
        best = dt if best is None else min(best, dt)
env = {k: v for k, v in os.environ.items() if k.startswith("MV_")}
print(f"e2e pinned {env}: best {best * 1e3:.3f} ms -> {n / best / 1e6:.1f} M/s ok={ok}", flush=True)
