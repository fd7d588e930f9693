#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_blocks.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r02k.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_r02k.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED|Error" gpurun_out/pytest_r02k.log | head -30; exit $rc; }
for qm in 0 4096 16384 65536; do
MV_REDUCE_QUAD=$qm timeout -k 10 200 python bench.py --cpu-sample 0 --no-e2e --steps 20 --sustain-repeats 0 --no-config4 --no-adversarial --streams 1 > gpurun_out/k_c2.json 2> gpurun_out/k_c2.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/k_c2.json')); print('c2 quadmax=$qm', round(d['value']/1e6,1), d['correct'], d['pipeline']['stage_ms'])"
done
