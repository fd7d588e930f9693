#!/bin/bash
# Online path: comb16 barrier inside the decode, hoisted-read hash: comb / block / ingest / engine
# tests, config-5 line, config-5 kernel stats.   tools/gpu_r03l.sh <tag>
set -o pipefail
TAG=${1:-r03l}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_comb.py tests/test_gpu_blocks.py tests/test_gpu_engine.py tests/test_gpu_ingest.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_$TAG.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED" gpurun_out/pytest_$TAG.log | head -30; exit $rc; }
timeout -k 10 200 python bench.py --workload config5 --cpu-sample 1 --batches 3000 --conc-seconds 2 > gpurun_out/c5_$TAG.json 2> gpurun_out/c5_$TAG.err || { tail -5 gpurun_out/c5_$TAG.err; exit 1; }
python - <<PY
import json
d=json.load(open("gpurun_out/c5_$TAG.json"))
for s,v in d["shapes"].items():
    c=v["concurrent_1_block_callers"]
    print(s, "gpu", v["gpu"]["p50_us"], v["gpu"]["p99_us"], "cpu16", v.get("cpu_16t",{}).get("p50_us"), v.get("cpu_16t",{}).get("p99_us"), "conc gpu", c["gpu"]["blocks_per_s"], c["gpu"]["p50_us"], "cpu", c.get("cpu_own_core",{}).get("blocks_per_s"))
PY
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/c5prof_$TAG -o run -f csv -- python bench.py --workload config5 --cpu-sample 0 --batches 1000 --conc-seconds 0.2 > gpurun_out/c5prof_$TAG.log 2>&1 || exit 1
python - <<PY
import csv
for r in csv.DictReader(open("gpurun_out/c5prof_$TAG/run_kernel_stats.csv")):
    print(r["Name"][:40], r["Calls"], round(float(r["AverageNs"])/1e3,1), "us avg", round(float(r["MinNs"])/1e3,1), "min")
PY
