#!/bin/bash
# Straight-line SHA-512: all GPU tests, chain microbench, config-5 line, comb phases, config-2
# and config-4 quick lines.   tools/gpu_r03h.sh <tag>
set -o pipefail
TAG=${1:-r03h}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_gpu_$TAG.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED" gpurun_out/pytest_gpu_$TAG.log | head -30; exit $rc; }
timeout -k 10 60 tools/microbench_chain > gpurun_out/chain_$TAG.jsonl 2>&1 || { cat gpurun_out/chain_$TAG.jsonl; exit 1; }
cat gpurun_out/chain_$TAG.jsonl
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
timeout -k 10 300 python bench.py --cpu-sample 0 --no-config5 --no-wal --no-adversarial --sustain-repeats 1 --config4-batch 1048576 > gpurun_out/c2_$TAG.json 2> gpurun_out/c2_$TAG.err || { tail -5 gpurun_out/c2_$TAG.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/c2_$TAG.json')); print('c2', round(d['value']/1e6,1), d['correct'], 'frac', d['roofline']['frac'], d['roofline']['stage_ms_one_stream']); c=d['config4']; print('c4', round(c['value']/1e6,1), c['pipeline']['stage_ms']); print('e2e', d['end_to_end']['value'])"
