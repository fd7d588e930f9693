#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_blocks.py tests/test_gpu_verify.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r02n.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_r02n.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED|Error" gpurun_out/pytest_r02n.log | head -30; exit $rc; }
for gg in 8 16; do
  MV_GUARD_GROUPS=$gg timeout -k 10 150 python bench.py --cpu-sample 0 --no-e2e --steps 20 --sustain-repeats 0 --no-config4 > gpurun_out/n_g$gg.json 2> gpurun_out/n_g$gg.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/n_g$gg.json')); a=d['adversarial']; print($gg, round(d['value']/1e6,1), d['correct'], [(k, round(v['value']/1e6,1), v['ratio_to_all_valid']) for k,v in a.items() if k!='note'])"
done
