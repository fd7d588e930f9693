#!/bin/bash
# comb16 with eight table roles: comb / block tests, phases, config-5 line; e2e first-batch split A/B.
#   tools/gpu_r03j.sh <tag>
set -o pipefail
TAG=${1:-r03j}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_comb.py tests/test_gpu_blocks.py tests/test_gpu_engine.py tests/test_gpu_verify.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_$TAG.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED" gpurun_out/pytest_$TAG.log | head -30; exit $rc; }
timeout -k 10 60 tools/comb_phase > gpurun_out/comb_phase_$TAG.jsonl 2>&1 || { cat gpurun_out/comb_phase_$TAG.jsonl; exit 1; }
cat gpurun_out/comb_phase_$TAG.jsonl
timeout -k 10 200 python bench.py --workload config5 --cpu-sample 0 --batches 2000 --conc-seconds 1 > gpurun_out/c5_$TAG.json 2> gpurun_out/c5_$TAG.err || { tail -5 gpurun_out/c5_$TAG.err; exit 1; }
python - <<PY
import json
d=json.load(open("gpurun_out/c5_$TAG.json"))
for s,v in d["shapes"].items():
    c=v["concurrent_1_block_callers"]["gpu"]
    print(s, v["gpu"]["p50_us"], v["gpu"]["p99_us"], "conc", c["blocks_per_s"], c["p50_us"], c["calls_per_device_pass"])
PY
for f in 0.5 0.6 0.7; do
  MV_STREAM_FIRST=$f timeout -k 10 120 python tools/pipe_probe.py > gpurun_out/e2e_f${f}_$TAG.log 2>&1 || { tail -5 gpurun_out/e2e_f${f}_$TAG.log; exit 1; }
  echo "first=$f: $(grep pinned gpurun_out/e2e_f${f}_$TAG.log)"
done
