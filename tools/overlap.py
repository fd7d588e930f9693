"""Busy time and overlap of two kernel classes in a rocprofv3 --kernel-trace CSV: how long kernels
matching A ran, how long kernels matching B ran, and how long both ran at once (union of each
class's intervals, then their intersection), over the last `window_ms` of the trace.
  python tools/overlap.py <trace_dir> <regexA> <regexB> [window_ms]
e.g. the config-4 walk against the verification kernels:
  python tools/overlap.py profiles/r06/trace_c4 k_block_walk 'k_bv_|k_part_|k_fine_|k_block_(digest|verdict)' 200"""
import csv
import glob
import re
import sys


def union(iv):
    out = []
    for s, e in sorted(iv):
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def intersect(a, b):
    i = j = 0
    tot = 0
    while i < len(a) and j < len(b):
        s, e = max(a[i][0], b[j][0]), min(a[i][1], b[j][1])
        if e > s:
            tot += e - s
        if a[i][1] < b[j][1]:
            i += 1
        else:
            j += 1
    return tot


def main():
    d, ra, rb = sys.argv[1], re.compile(sys.argv[2]), re.compile(sys.argv[3])
    window_ms = float(sys.argv[4]) if len(sys.argv) > 4 else 200.0
    ev = []
    for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    end = max(e for _, e, _ in ev)
    t0 = end - window_ms * 1e6
    clip = lambda s, e: (max(s, t0), e)
    a = union([clip(s, e) for s, e, n in ev if e > t0 and ra.search(n)])
    b = union([clip(s, e) for s, e, n in ev if e > t0 and rb.search(n)])
    busy = lambda iv: sum(e - s for s, e in iv) / 1e6
    both = intersect(a, b) / 1e6
    print(f"window {window_ms:.0f} ms (trace end - window .. end)")
    print(f"A /{sys.argv[2]}/ busy {busy(a):.1f} ms")
    print(f"B /{sys.argv[3]}/ busy {busy(b):.1f} ms")
    print(f"A and B at once {both:.1f} ms; either {busy(a) + busy(b) - both:.1f} ms")


if __name__ == "__main__":
    main()
