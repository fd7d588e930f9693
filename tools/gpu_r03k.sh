#!/bin/bash
# comb16 / k_comb_post at 4 signatures per workgroup: comb / block tests, phases, config-5 line.
#   tools/gpu_r03k.sh <tag>
set -o pipefail
TAG=${1:-r03k}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_comb.py tests/test_gpu_blocks.py tests/test_gpu_engine.py tests/test_gpu_verify.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_$TAG.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED" gpurun_out/pytest_$TAG.log | head -30; exit $rc; }
timeout -k 10 60 tools/comb_phase > gpurun_out/comb_phase_$TAG.jsonl 2>&1 || { cat gpurun_out/comb_phase_$TAG.jsonl; exit 1; }
cat gpurun_out/comb_phase_$TAG.jsonl
timeout -k 10 200 python bench.py --workload config5 --cpu-sample 1 --batches 3000 --conc-seconds 2 > gpurun_out/c5_$TAG.json 2> gpurun_out/c5_$TAG.err || { tail -5 gpurun_out/c5_$TAG.err; exit 1; }
python - <<PY
import json
d=json.load(open("gpurun_out/c5_$TAG.json"))
for s,v in d["shapes"].items():
    c=v["concurrent_1_block_callers"]
    print(s, "gpu", v["gpu"]["p50_us"], v["gpu"]["p99_us"], "cpu16", v.get("cpu_16t",{}).get("p50_us"), v.get("cpu_16t",{}).get("p99_us"), "conc gpu", c["gpu"]["blocks_per_s"], c["gpu"]["p50_us"], "cpu", c.get("cpu_own_core",{}).get("blocks_per_s"))
PY
