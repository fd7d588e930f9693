"""Teardown probe: the host-fed config-4 leg's allocation pattern -- a
mv_host_alloc caller buffer DMA'd in place then host_free'd, a pageable pass, a torch pinned
tensor -- then normal interpreter exit. /proc/self/maps is written at exit (before the C++
static destructors run), so a crash PC printed by a signal handler can be mapped to its library.

    python tools/teardown_probe.py <maps-out>
"""
import atexit
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    maps_out = sys.argv[1]
    atexit.register(lambda: open(maps_out, "w").write(open("/proc/self/maps").read()))
    import torch

    import bench_blocks
    import mysticeti_amd as M
    import mysticeti_amd.blocks as MB

    torch.cuda.set_device(0)
    eng = M.Engine(devices=(0,))
    base = MB.config4(eng, rounds=41)
    pks, stakes = MB.committee(eng, 100, distinct=True)
    eng.set_committee(pks, stakes, 0)
    buf, off, ln = MB.pack(base)
    nb = len(base)
    span = (int(off[-1] + ln[-1]) + 7) & ~7
    r = bench_blocks.config4_host_fed(eng, torch, torch.device("cuda", 0), buf, off, ln, nb, span, 1 << 16, calls=2)
    print("host_fed", r["value"], r["correct"], flush=True)
    eng.close()
    print("closed", flush=True)


if __name__ == "__main__":
    main()
