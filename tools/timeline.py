"""Prints a compact timeline (kernels and memory copies, start/end in us relative to a window)
from rocprofv3 --kernel-trace --memory-copy-trace CSV output. Usage:
  python tools/timeline.py <out_dir> [last_ms]   (the last `last_ms` milliseconds of activity)"""
import csv, glob, sys

d = sys.argv[1]
last_ms = float(sys.argv[2]) if len(sys.argv) > 2 else 8.0
ev = []
for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K", r["Kernel_Name"][:40], r.get("Stream_Id", r.get("Queue_Id", ""))))
for f in glob.glob(f"{d}/**/*memory_copy_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "C", r.get("Direction", "copy"), r.get("Stream_Id", r.get("Queue_Id", ""))))
ev.sort()
end = max(e[1] for e in ev)
t0 = end - last_ms * 1e6
sel = [e for e in ev if e[1] >= t0]
base = sel[0][0]
for s, e, k, name, q in sel:
    print(f"{(s - base) / 1e3:9.1f} {(e - base) / 1e3:9.1f} {(e - s) / 1e3:8.1f} {k} q{q:>3} {name}")
