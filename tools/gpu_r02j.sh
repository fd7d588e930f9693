#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_blocks.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r02j.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_r02j.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED|Error" gpurun_out/pytest_r02j.log | head -30; exit $rc; }
timeout -k 10 200 python bench.py --cpu-sample 0 --no-e2e --steps 20 --sustain-repeats 3 --no-config4 > gpurun_out/j_c2.json 2> gpurun_out/j_c2.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/j_c2.json')); print('c2', round(d['value']/1e6,1), round(d['sustained']['median']/1e6,1), d['correct'], d['roofline']['stage_ms_one_stream'], [(k, round(v['value']/1e6,1), v['ratio_to_all_valid']) for k,v in d['adversarial'].items() if k!='note'])"
timeout -k 10 200 python bench.py --workload config4 --cpu-sample 0 --steps 20 > gpurun_out/j_c4.json 2> gpurun_out/j_c4.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/j_c4.json')); print('c4', round(d['value']/1e6,2), d['correct'], d['pipeline']['stage_ms'])"
