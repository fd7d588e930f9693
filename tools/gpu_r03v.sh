#!/bin/bash
# Ingest folded into k_verify_comb16: block / ingest / engine / comb tests, config-5 line
# (ingest in comb vs a separate k_block_ingest, 2 interleaved reps), then config-4 ingest LDS pad A/B.
set -o pipefail
TAG=${1:-r03v}
mkdir -p gpurun_out/c4pad
timeout -k 10 600 python -u -m pytest tests/test_gpu_ingest.py tests/test_gpu_blocks.py tests/test_gpu_engine.py tests/test_gpu_comb.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_$TAG.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED" gpurun_out/pytest_$TAG.log | head -30; exit $rc; }
for rep in 1 2; do
for g in 1 0; do
  MV_INGEST_IN_COMB=$g timeout -k 10 200 python bench.py --workload config5 --cpu-sample 0 --batches 2000 --conc-seconds 2 > gpurun_out/c5_g${g}_${rep}_$TAG.json 2> gpurun_out/c5_g${g}_${rep}_$TAG.err || { tail -5 gpurun_out/c5_g${g}_${rep}_$TAG.err; exit 1; }
  python - <<PY
import json
d=json.load(open("gpurun_out/c5_g${g}_${rep}_$TAG.json"))
v=d["shapes"]["config1"]; c=v["concurrent_1_block_callers"]["gpu"]; w=d["shapes"]["config4"]; c4=w["concurrent_1_block_callers"]["gpu"]
print("rep $rep ingest_in_comb=$g c1 64-blk p50", v["gpu"]["p50_us"], v["gpu"]["p99_us"], "conc", c["blocks_per_s"], c["p50_us"], "| c4 64-blk", w["gpu"]["p50_us"], "conc", c4["blocks_per_s"])
PY
done
done
for pad in 0 12288 0 12288; do
  MV_INGEST_LDS_PAD=$pad timeout -k 10 300 python bench.py --workload config4 --steps 20 --warmup 3 --cpu-sample 0 --host-fed-blocks 0 > gpurun_out/c4pad/$pad.json 2> gpurun_out/c4pad/$pad.err || { tail -5 gpurun_out/c4pad/$pad.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/c4pad/$pad.json')); print('pad $pad', round(d['value']/1e6,2), d['correct'], d['pipeline']['stage_ms_as_run']['parse'], d['pipeline']['stage_ms_as_run']['hash'])"
done
