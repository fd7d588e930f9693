#!/bin/bash
# In-place DMA of pinned block buffers: block / engine tests, host-fed config 4 (pinned and pageable).
set -o pipefail
TAG=${1:-r03s}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_blocks.py tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_$TAG.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED" gpurun_out/pytest_$TAG.log | head -30; exit $rc; }
MV_BLK_TRACE=1 timeout -k 10 300 python bench.py --workload config4 --batch 262144 --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/c4hf_$TAG.json 2> gpurun_out/c4hf_$TAG.err || { tail -5 gpurun_out/c4hf_$TAG.err; exit 1; }
python3 - <<PY
import json
d=json.load(open("gpurun_out/c4hf_$TAG.json")); h=d["host_fed"]
print("pinned", h["value"], h["frac_of_pcie_bound"], "pageable", h["pageable"], "h2d", h["h2d_GBps_pinned"], h["correct"])
PY
grep "in place" gpurun_out/c4hf_$TAG.err | tail -3
