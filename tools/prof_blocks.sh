#!/bin/bash
# rocprofv3 kernel trace of the block benches (single stream, so per-kernel times are clean)
#   tools/prof_blocks.sh <tag>
set -o pipefail
TAG=${1:-blk}
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG/c4 -o run -- \
  python bench.py --workload config4 --batch ${C4_BATCH:-262144} --steps 3 --warmup 1 --streams 1 --cpu-sample 0 \
  > gpurun_out/prof_$TAG/c4.log 2>&1 || { tail -20 gpurun_out/prof_$TAG/c4.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG/c5 -o run -- \
  python bench.py --workload config5 --batches 2000 --cpu-sample 0 \
  > gpurun_out/prof_$TAG/c5.log 2>&1 || { tail -20 gpurun_out/prof_$TAG/c5.log; exit 1; }
python - <<PY
import csv, glob
for w in ("c4", "c5"):
    for f in glob.glob(f"gpurun_out/prof_$TAG/{w}/**/*kernel_stats.csv", recursive=True):
        print("==", w, f)
        for r in csv.DictReader(open(f)):
            print(f"{r['Name'][:60]:60s} {r['Calls']:>7s} {float(r['AverageNs'])/1e3:10.1f} us")
PY
