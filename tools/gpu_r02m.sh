#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
for g in 8 16; do
  MV_BV_SEG=1 timeout -k 10 150 python bench.py --cpu-sample 0 --no-e2e --steps 20 --sustain-repeats 0 --no-config4 --no-adversarial --streams 1 --groups $g > gpurun_out/m_s1_$g.json 2> gpurun_out/m_s1_$g.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/m_s1_$g.json')); print('seg1 1 stream g$g', round(d['value']/1e6,1), d['pipeline']['stage_ms'])"
done
for gg in 8 16; do
  MV_BV_SEG=1 MV_GUARD_GROUPS=$gg timeout -k 10 150 python bench.py --cpu-sample 0 --no-e2e --steps 20 --sustain-repeats 0 --no-config4 > gpurun_out/m_g$gg.json 2> gpurun_out/m_g$gg.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/m_g$gg.json')); a=d['adversarial']; print('seg1', $gg, round(d['value']/1e6,1), d['correct'], [(k, round(v['value']/1e6,1), v['ratio_to_all_valid']) for k,v in a.items() if k!='note'])"
done
