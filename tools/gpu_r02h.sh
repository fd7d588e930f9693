#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_primitives.py tests/test_gpu_blocks.py tests/test_gpu_ingest.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r02h.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_r02h.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED|Error" gpurun_out/pytest_r02h.log | head -30; exit $rc; }
timeout -k 10 200 python bench.py --workload config4 --cpu-sample 0 --steps 20 > gpurun_out/h_c4.json 2> gpurun_out/h_c4.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/h_c4.json')); print('c4', round(d['value']/1e6,2), d['correct'], d['pipeline']['stage_ms'])"
