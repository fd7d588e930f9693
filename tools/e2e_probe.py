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
# (batches, batches with a failed equation, sub-batch equations, failed ones): all-valid inputs
# must never fail an equation
print(f"batch counters after the single calls: {eng.batch_counters()}", flush=True)

# two callers at once (MV_PROBE_TWO=1): each thread its own pinned copy; per-call start/end
# relative to the pair's start, so a timeline of the same run shows what each call waited for
if os.environ.get("MV_PROBE_TWO"):
    import threading

    pm2, ps2, pp2 = eng.host_empty(msg.shape), eng.host_empty(sig.shape), eng.host_empty(pk.shape)
    pm2[:], ps2[:], pp2[:] = msg, sig, pk
    for it in range(4):
        marks = [None, None]
        t0 = time.perf_counter()

        def call(c, a):
            s = time.perf_counter()
            st2 = eng.ed25519_verify(*a)
            marks[c] = (s - t0, time.perf_counter() - t0, bool((st2 == 0).all()))

        th = [threading.Thread(target=call, args=(c, a)) for c, a in enumerate(((pm, ps, pp), (pm2, ps2, pp2)))]
        for x in th:
            x.start()
        for x in th:
            x.join()
        dt = time.perf_counter() - t0
        print(f"counters {eng.batch_counters()}; two callers: {dt * 1e3:.3f} ms -> {2 * n / dt / 1e6:.1f} M/s; calls (start, end ms, ok): "
              + ", ".join(f"({m[0] * 1e3:.2f}, {m[1] * 1e3:.2f}, {m[2]})" for m in marks), flush=True)
