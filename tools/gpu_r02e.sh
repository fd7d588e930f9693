#!/bin/bash
# batch/block/engine GPU tests, then config-4 with and without the per-key A term
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_blocks.py tests/test_gpu_engine.py tests/test_gpu_ingest.py tests/test_gpu_comb.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_r02e.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_r02e.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED|Error" gpurun_out/pytest_r02e.log | head -30; exit $rc; }
for v in 1 0; do
  MV_NO_KEY_AGG=$v timeout -k 10 200 python bench.py --workload config4 --cpu-sample 0 --steps 20 > gpurun_out/c4_agg$v.json 2> gpurun_out/c4_agg$v.err || { tail gpurun_out/c4_agg$v.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/c4_agg$v.json')); print('no_agg=$v', round(d['value']/1e6,2), d['correct'], d['pipeline']['stage_ms'])"
done
MV_NO_KEY_AGG=0 timeout -k 10 200 python bench.py --workload config4 --cpu-sample 0 --steps 20 --streams 1 > gpurun_out/c4_s1.json 2> gpurun_out/c4_s1.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/c4_s1.json')); print('1 stream', round(d['value']/1e6,2), d['correct'], d['pipeline']['stage_ms'])"
