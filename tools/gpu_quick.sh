#!/bin/bash
# Quick A/B on the GPU box: GPU tests, config-2 and config-4 bench lines (no CPU legs).
#   tools/gpu_quick.sh <tag> [pytest selection]
set -o pipefail
TAG=${1:-q}; SEL=${2:-tests}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest $SEL -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_$TAG.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED|Error" gpurun_out/pytest_$TAG.log | head -30; exit $rc; }
timeout -k 10 200 python bench.py --cpu-sample 0 --no-e2e --sustain-repeats 0 --no-adversarial --no-config4 > gpurun_out/${TAG}_c2.json 2> gpurun_out/${TAG}_c2.err || exit 1
timeout -k 10 300 python bench.py --workload config4 --cpu-sample 0 > gpurun_out/${TAG}_c4.json 2> gpurun_out/${TAG}_c4.err || exit 1
python - <<PY
import json
d=json.load(open("gpurun_out/${TAG}_c2.json")); r=d["roofline"]
print("c2", round(d["value"]/1e6,1), "M/s", d["correct"], r["stage_ms_one_stream"])
d=json.load(open("gpurun_out/${TAG}_c4.json")); d=d.get("config4") or d
print("c4", round(d["value"]/1e6,1), "M/s", d["correct"], d["pipeline"]["stage_ms"])
PY
