#!/bin/bash
# A/B of an experiment build against the product build on config 4 (and config 2):
#   tools/gpu_ab.sh <tag> <variant> [workload]
set -o pipefail
TAG=$1; VAR=$2; WL=${3:-config4}
mkdir -p gpurun_out/$TAG
for run in base var base var; do
  if [ $run = var ]; then export MV_LIB=mysticeti_amd/_build/$VAR/libmysti_verify.so; else unset MV_LIB; fi
  timeout -k 10 300 python bench.py --workload $WL --cpu-sample 0 --no-e2e --sustain-repeats 0 --no-adversarial --no-config4 > gpurun_out/$TAG/$run.json 2> gpurun_out/$TAG/$run.err || exit 1
  python - <<PY
import json
d=json.load(open("gpurun_out/$TAG/$run.json")); d=d.get("config4") if "$WL"=="config4" and d.get("config4") else d
st=d.get("pipeline",{}).get("stage_ms") or d.get("roofline",{}).get("stage_ms_one_stream")
print("$run", round(d["value"]/1e6,2), "M/s", d["correct"], st)
PY
done
