#!/bin/bash
# Fused ingest+hash check: block GPU tests, then config-4 throughput fused vs two-kernel.
#   tools/gpu_fused.sh <tag>
set -o pipefail
TAG=${1:-fz}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_ingest.py tests/test_gpu_blocks.py tests/test_gpu_engine.py tests/test_gpu_comb.py tests/test_gpu_primitives.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_fused_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_fused_$TAG.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED|Error" gpurun_out/pytest_fused_$TAG.log | head -30; exit $rc; }
timeout -k 10 300 python bench.py --workload config4 --steps 20 --warmup 3 --cpu-sample 0 > gpurun_out/c4_fused_$TAG.json 2> gpurun_out/c4_fused_$TAG.err || { tail -5 gpurun_out/c4_fused_$TAG.err; exit 1; }
MV_BLK_FUSED=0 timeout -k 10 300 python bench.py --workload config4 --steps 20 --warmup 3 --cpu-sample 0 > gpurun_out/c4_old_$TAG.json 2> gpurun_out/c4_old_$TAG.err || { tail -5 gpurun_out/c4_old_$TAG.err; exit 1; }
python - <<PY
import json
for k in ("fused","old"):
    d=json.load(open(f"gpurun_out/c4_{k}_$TAG.json"))
    print(k, round(d["value"]/1e6,2), d["correct"], d["pipeline"]["stage_ms"])
PY
