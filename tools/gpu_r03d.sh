#!/bin/bash
# Block-path GPU tests, config-5 latency with 2 vs 4 pass sets in flight, config 4 with the
# host-fed leg.   tools/gpu_r03d.sh <tag>
set -o pipefail
TAG=${1:-r03d}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_ingest.py tests/test_gpu_blocks.py tests/test_gpu_engine.py tests/test_gpu_comb.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_blk_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_blk_$TAG.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED|Error" gpurun_out/pytest_blk_$TAG.log | head -30; exit $rc; }
for k in 2 4; do
  MV_PASS_SETS=$k timeout -k 10 200 python bench.py --workload config5 --cpu-sample 0 --batches 2000 --conc-seconds 1 > gpurun_out/c5_ps${k}_$TAG.json 2> gpurun_out/c5_ps${k}_$TAG.err || { tail -5 gpurun_out/c5_ps${k}_$TAG.err; exit 1; }
done
python - <<PY
import json
for k in (2, 4):
    d=json.load(open(f"gpurun_out/c5_ps{k}_$TAG.json"))
    for s,v in d["shapes"].items():
        c=v["concurrent_1_block_callers"]["gpu"]
        print("sets", k, s, v["gpu"]["p50_us"], v["gpu"]["p99_us"], "conc", c["blocks_per_s"], c["p50_us"], c["calls_per_device_pass"])
PY
timeout -k 10 400 python bench.py --workload config4 --batch 1048576 --steps 20 --warmup 3 --cpu-sample 0 > gpurun_out/c4_$TAG.json 2> gpurun_out/c4_$TAG.err || { tail -5 gpurun_out/c4_$TAG.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/c4_$TAG.json')); print('c4', round(d['value']/1e6,2), d['correct'], d['pipeline']['stage_ms']); print(json.dumps(d['host_fed']))"
