#!/bin/bash
# config-4 bench + kernel trace only (quick iteration on the block pipeline)
set -o pipefail
TAG=${1:-c4}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ingest.py tests/test_gpu_blocks.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pt_$TAG.log 2>&1 || { tail -30 gpurun_out/pt_$TAG.log; exit 1; }
tail -1 gpurun_out/pt_$TAG.log
timeout -k 10 300 python bench.py --workload config4 --batch ${C4_BATCH:-1048576} --steps 10 --warmup 2 --cpu-sample 0 > gpurun_out/c4_$TAG.json 2> gpurun_out/c4_$TAG.err || { tail -20 gpurun_out/c4_$TAG.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/c4_$TAG.json')); print(d['value'], d['ms_per_step'], d['correct'], d['pipeline']['stage_ms'], d['roofline']['frac'])"
