"""Top kernels of a rocprofv3 --kernel-trace --stats run (tools/gpu.sh trace:W)."""
import csv
import glob
import sys

for f in glob.glob(f"{sys.argv[1]}/**/*kernel_stats.csv", recursive=True):
    rows = sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))
    for r in rows[:int(sys.argv[2]) if len(sys.argv) > 2 else 12]:
        print(f"{r['Name'][:60]:60s} calls={r['Calls']:>6s} avg_us={float(r['AverageNs']) / 1e3:10.1f} "
              f"pct={float(r['Percentage']):5.1f}")
