#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_verify.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r02o.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_r02o.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED|Error" gpurun_out/pytest_r02o.log | head -30; exit $rc; }
for v in 1 0; do
MV_NO_PIPELINE=$([ $v = 1 ] && echo 1) timeout -k 10 150 python bench.py --cpu-sample 0 --steps 20 --sustain-repeats 0 --no-config4 --no-adversarial > gpurun_out/o_$v.json 2> gpurun_out/o_$v.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/o_$v.json')); print('nopipe=$v', round(d['value']/1e6,1), d['correct'], d['end_to_end'])"
done
