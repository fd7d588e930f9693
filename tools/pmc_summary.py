"""Summarise rocprofv3 --pmc CSVs for one kernel: per-dispatch averages + derived metrics.

    python tools/pmc_summary.py gpurun_out/prof_<tag> [kernel-substring] [--json out.json]

--json writes {"kernel", "hbm_bytes_per_launch", "fetch_bytes", "write_bytes", counters...}:
HBM bytes per launch = 2 x FETCH_SIZE (gfx950 tallies 128-B requests at 64 B,
MI355X_MICROARCH.md HBM section; Infinity-Cache hits are counted too) + WRITE_SIZE, KiB -> B.
bench.py reads it for roofline.traffic.
"""
import collections
import csv
import glob
import sys

args = [a for a in sys.argv[1:]]
jout = None
if "--json" in args:
    i = args.index("--json")
    jout = args[i + 1]
    del args[i:i + 2]
d = args[0]
kname = args[1] if len(args) > 1 else "k_verify"
agg = collections.defaultdict(lambda: collections.defaultdict(float))
meta = {}
for f in sorted(glob.glob(f"{d}/pmc*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if kname not in r["Kernel_Name"]:
            continue
        agg[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
        meta = {k: r[k] for k in ("Grid_Size", "Workgroup_Size", "VGPR_Count", "Accum_VGPR_Count", "SGPR_Count",
                                   "LDS_Block_Size", "Scratch_Size")}
avg = {c: sum(v.values()) / len(v) for c, v in agg.items()}
print(f"# {kname}: per-dispatch averages from {d}")
print("#", meta)
for c in sorted(avg):
    print(f"{c:28s} {avg[c]:.4e}")
dur = None
for f in glob.glob(f"{d}/trace1/*kernel_stats.csv") or glob.glob(f"{d}/trace/*kernel_stats.csv"):
    for r in csv.DictReader(open(f)):
        if kname in r["Name"]:
            dur = float(r["AverageNs"]) * 1e-9
if dur:
    print(f"{'kernel_avg_s':28s} {dur:.6e}")
    waves = avg.get("SQ_WAVES", 0)
    if "GRBM_GUI_ACTIVE" in avg:
        clk = avg["GRBM_GUI_ACTIVE"] / 8 / dur
        print(f"{'effective_clock_GHz':28s} {clk / 1e9:.3f}")
        simd_cycles = 1024 * avg["GRBM_GUI_ACTIVE"] / 8
        if "SQ_INSTS_VALU" in avg:
            slots = avg["SQ_INSTS_VALU"] + avg.get("SQ_INSTS_VALU_INT64", 0)  # 64-bit ops issue at half rate
            print(f"{'valu_issue_util':28s} {2 * slots / simd_cycles:.3f}  (2 cyc/full-rate wave-instr, INT64 x2)")
    if waves and "SQ_INSTS_VALU" in avg:
        print(f"{'valu_instr_per_wave':28s} {avg['SQ_INSTS_VALU'] / waves:.4e}")
    if "SQ_WAVE_CYCLES" in avg:
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if k in avg:
                print(f"{k + '_frac':28s} {avg[k] / avg['SQ_WAVE_CYCLES']:.3f}")
    if "FETCH_SIZE" in avg:
        print(f"{'fetch_GBps (x2 gfx950 corr)':28s} {2 * avg['FETCH_SIZE'] * 1024 / dur / 1e9:.1f}")
    if "WRITE_SIZE" in avg:
        print(f"{'write_GBps':28s} {avg['WRITE_SIZE'] * 1024 / dur / 1e9:.1f}")

if jout:
    import json

    fetch = 2 * avg["FETCH_SIZE"] * 1024 if "FETCH_SIZE" in avg else None
    write = avg["WRITE_SIZE"] * 1024 if "WRITE_SIZE" in avg else None
    out = {"kernel": kname, "source": d, "hbm_bytes_per_launch": (fetch or 0) + (write or 0) if fetch is not None else None,
           "fetch_bytes": fetch, "write_bytes": write, "meta": meta, "counters": avg}
    json.dump(out, open(jout, "w"), indent=1)
