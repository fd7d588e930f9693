#!/bin/bash
# round-2 iteration: batch/block GPU tests, then the grouped-equation A/B on config 2
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_blocks.py -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_r02a.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_r02a.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED|Error" gpurun_out/pytest_r02a.log | head -30; exit $rc; }
for cfg in "--groups 1" "--groups 4" "--groups 8" "--groups 16" "--corrupt 1" "--corrupt 1 --groups 8" "--corrupt 1 --groups 16" "--corrupt 10486"; do
  tag=$(echo $cfg | tr -d ' -')
  timeout -k 10 120 python bench.py --cpu-sample 0 --no-e2e --steps 40 $cfg > gpurun_out/b_$tag.json 2> gpurun_out/b_$tag.err || { cat gpurun_out/b_$tag.err | tail; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/b_$tag.json')); print('$cfg', round(d['value']/1e6,1), d['correct'], d['roofline']['isolated']['stage_ms'] if d['roofline'].get('isolated') else '')"
done
