#!/bin/bash
# Config-4 fused vs two-kernel throughput on one box, then the config-5 kernel timeline.
#   tools/gpu_r03b.sh <tag>
set -o pipefail
TAG=${1:-r03b}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for k in old fused; do
  if [ $k = old ]; then export MV_BLK_FUSED=0; else unset MV_BLK_FUSED; fi
  timeout -k 10 300 python bench.py --workload config4 --steps 20 --warmup 3 --cpu-sample 0 > gpurun_out/c4_${k}_$TAG.json 2> gpurun_out/c4_${k}_$TAG.err || { tail -5 gpurun_out/c4_${k}_$TAG.err; exit 1; }
done
unset MV_BLK_FUSED
python - <<PY
import json
for k in ("old","fused"):
    d=json.load(open(f"gpurun_out/c4_{k}_$TAG.json"))
    print(k, round(d["value"]/1e6,2), d["correct"], d["pipeline"]["stage_ms"])
PY
timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/c5tl_$TAG -o run -f csv -- python bench.py --workload config5 --cpu-sample 0 --batches 500 --conc-seconds 0.2 > gpurun_out/c5tl_$TAG.log 2>&1 || exit 1
python tools/timeline.py gpurun_out/c5tl_$TAG 3 > gpurun_out/c5_timeline_$TAG.txt
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/c4prof_$TAG -o run -f csv -- python bench.py --workload config4 --steps 10 --warmup 2 --cpu-sample 0 > gpurun_out/c4prof_$TAG.log 2>&1 || exit 1
echo done
