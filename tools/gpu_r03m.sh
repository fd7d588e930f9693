#!/bin/bash
# Concurrent 1-block callers: pass sets 2 / 3 / 4, event wait blocking vs polled.
#   tools/gpu_r03m.sh <tag>
set -o pipefail
TAG=${1:-r03m}
mkdir -p gpurun_out
for ps in 2 3 4; do
  for sp in 0 1; do
    MV_PASS_SETS=$ps MV_PASS_SPIN=$sp timeout -k 10 200 python bench.py --workload config5 --cpu-sample 0 --batches 1000 --conc-seconds 2 > gpurun_out/c5_${ps}_${sp}_$TAG.json 2> gpurun_out/c5_${ps}_${sp}_$TAG.err || { tail -5 gpurun_out/c5_${ps}_${sp}_$TAG.err; exit 1; }
    python - <<PY
import json
d=json.load(open("gpurun_out/c5_${ps}_${sp}_$TAG.json"))
v=d["shapes"]["config1"]; c=v["concurrent_1_block_callers"]["gpu"]
w=d["shapes"]["config4"]; c4=w["concurrent_1_block_callers"]["gpu"]
print("sets $ps spin $sp: c1 64-blk p50", v["gpu"]["p50_us"], "conc", c["blocks_per_s"], c["p50_us"], c["calls_per_device_pass"], "| c4 64-blk", w["gpu"]["p50_us"], "conc", c4["blocks_per_s"])
PY
  done
done
