#!/bin/bash
# in-place ingest: block tests, then config 4 (quad hash vs lane hash)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ingest.py tests/test_gpu_blocks.py tests/test_gpu_engine.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r02g.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_r02g.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED|Error" gpurun_out/pytest_r02g.log | head -30; exit $rc; }
for h in 0 1; do
  MV_HASH_LANE=$h timeout -k 10 200 python bench.py --workload config4 --cpu-sample 0 --steps 20 > gpurun_out/g_c4_$h.json 2> gpurun_out/g_c4_$h.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/g_c4_$h.json')); print('hash_lane=$h', round(d['value']/1e6,2), d['correct'], d['pipeline']['stage_ms'])"
done
