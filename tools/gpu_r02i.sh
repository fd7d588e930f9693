#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_primitives.py tests/test_gpu_blocks.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r02i.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_r02i.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED|Error" gpurun_out/pytest_r02i.log | head -30; exit $rc; }
MV_B2Q_NS=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_blocks.py tests/test_gpu_primitives.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r02i2.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_r02i2.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED|Error" gpurun_out/pytest_r02i2.log | head -30; exit $rc; }
for ns in 1 2; do
  MV_B2Q_NS=$ns timeout -k 10 200 python bench.py --workload config4 --cpu-sample 0 --steps 20 > gpurun_out/i_c4_$ns.json 2> gpurun_out/i_c4_$ns.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/i_c4_$ns.json')); print('ns=$ns', round(d['value']/1e6,2), d['correct'], d['pipeline']['stage_ms']['hash'], d['pipeline']['stage_ms']['parse'])"
done
