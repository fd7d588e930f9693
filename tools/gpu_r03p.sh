#!/bin/bash
# Hash folded into k_verify_comb16: block / ingest / engine / comb tests, config-5 line (in-comb vs separate hash).
set -o pipefail
TAG=${1:-r03p}
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_ingest.py tests/test_gpu_blocks.py tests/test_gpu_engine.py tests/test_gpu_comb.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_$TAG.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED" gpurun_out/pytest_$TAG.log | head -30; exit $rc; }
for h in 1 0; do
  MV_HASH_IN_COMB=$h timeout -k 10 200 python bench.py --workload config5 --cpu-sample 0 --batches 2000 --conc-seconds 2 > gpurun_out/c5_h${h}_$TAG.json 2> gpurun_out/c5_h${h}_$TAG.err || { tail -5 gpurun_out/c5_h${h}_$TAG.err; exit 1; }
  python - <<PY
import json
d=json.load(open("gpurun_out/c5_h${h}_$TAG.json"))
v=d["shapes"]["config1"]; c=v["concurrent_1_block_callers"]["gpu"]; w=d["shapes"]["config4"]; c4=w["concurrent_1_block_callers"]["gpu"]
print("hash_in_comb=$h c1 64-blk p50", v["gpu"]["p50_us"], v["gpu"]["p99_us"], "conc", c["blocks_per_s"], c["p50_us"], "| c4 64-blk", w["gpu"]["p50_us"], "conc", c4["blocks_per_s"])
PY
done
