#!/bin/bash
# bucket segments x groups A/B (one stream), then adversarial rates per guard size
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_r02c.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_r02c.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED|Error" gpurun_out/pytest_r02c.log | head -30; exit $rc; }
for cfg in "1 1" "4 1" "4 4" "8 1" "8 8" "16 1" "16 16" "16 8" "16 32"; do
  set -- $cfg
  MV_BV_SEG=$2 timeout -k 10 120 python bench.py --cpu-sample 0 --no-e2e --steps 20 --sustain-repeats 0 --streams 1 --no-adversarial --groups $1 > gpurun_out/m_$1_$2.json 2> gpurun_out/m_$1_$2.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/m_$1_$2.json')); print('g$1 seg$2', round(d['value']/1e6,1), d['correct'], {k: round(v,3) for k,v in d['pipeline']['stage_ms'].items()})"
done
for gg in 8 16; do
  MV_GUARD_GROUPS=$gg timeout -k 10 120 python bench.py --cpu-sample 0 --no-e2e --steps 20 --sustain-repeats 0 > gpurun_out/adv2_g$gg.json 2> gpurun_out/adv2_g$gg.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/adv2_g$gg.json')); a=d['adversarial']; print($gg, round(d['value']/1e6,1), d['correct'], [(k, round(v['value']/1e6,1), v['ratio_to_all_valid']) for k,v in a.items() if k!='note'])"
done
