#!/bin/bash
# hash LDS padding + 128-B point records: tests, then A/B config 2 (pt128 vs pt112) and config 4
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_blocks.py tests/test_gpu_primitives.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r02f.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_r02f.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED|Error" gpurun_out/pytest_r02f.log | head -30; exit $rc; }
for v in "" "mysticeti_amd/_build/pt112/libmysti_verify.so"; do
  MV_LIB=$v timeout -k 10 200 python bench.py --cpu-sample 0 --no-e2e --steps 20 --sustain-repeats 3 --no-adversarial --no-config4 > gpurun_out/f_c2.json 2> gpurun_out/f_c2.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/f_c2.json')); print('lib=$v', round(d['value']/1e6,1), round(d['sustained']['median']/1e6,1), d['correct'], d['roofline']['stage_ms_one_stream'])"
done
timeout -k 10 200 python bench.py --workload config4 --cpu-sample 0 --steps 20 > gpurun_out/f_c4.json 2> gpurun_out/f_c4.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/f_c4.json')); print('c4', round(d['value']/1e6,2), d['correct'], d['pipeline']['stage_ms'])"
