"""CPU: the bench line's roofline.traffic comes from committed PMC summaries under profiles/,
which must travel to the GPU box (the driver runs bench.py there from the snapshot)."""
import fnmatch
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def test_pmc_summaries_found_for_every_headline_kernel():
    from bench import pmc_traffic

    for kernel, wl in (("k_bv_prep", "c2"), ("k_b2_lane", "c4"), ("k_wal_crc", "wal")):
        traffic, src = pmc_traffic(kernel, wl)
        assert traffic and traffic > 0, (kernel, src)
        assert src.startswith("profiles" + os.sep), src


def test_profiles_are_not_left_off_the_gpu_snapshot():
    pats = [p.strip() for p in open(os.path.join(ROOT, ".gpurunignore")) if p.strip()]
    for f in ("profiles/r05/pmc/pmc_c2_k_bv_prep.json", "profiles/r05/pmc/pmc_c4_k_b2_lane.json"):
        for p in pats:
            anchored = p.startswith("./")
            pat = p[2:] if anchored else p
            hits = fnmatch.fnmatch(f, pat) or f.startswith(pat.rstrip("/") + "/") if anchored else \
                any(fnmatch.fnmatch(part, pat) for part in f.split("/"))
            assert not hits, (f, p)
