#!/bin/bash
# guard-group A/B on the adversarial rates (one bad signature per 2^20, 1% corrupted)
set -o pipefail
mkdir -p gpurun_out
for gg in 4 8 16; do
  MV_GUARD_GROUPS=$gg timeout -k 10 120 python bench.py --cpu-sample 0 --no-e2e --steps 20 --sustain-repeats 0 > gpurun_out/adv_g$gg.json 2> gpurun_out/adv_g$gg.err || { tail gpurun_out/adv_g$gg.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/adv_g$gg.json')); a=d['adversarial']; print($gg, round(d['value']/1e6,1), d['correct'], [(k, round(v['value']/1e6,1), v['ratio_to_all_valid'], v['groups_per_batch'], v['groups_reverified_per_batch']) for k,v in a.items() if k!='note'])"
done
for gg in 1 4 8 16; do
  timeout -k 10 120 python bench.py --cpu-sample 0 --no-e2e --steps 20 --sustain-repeats 0 --streams 1 --no-adversarial --groups $gg > gpurun_out/s1_g$gg.json 2> gpurun_out/s1_g$gg.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/s1_g$gg.json')); print('1stream g$gg', round(d['value']/1e6,1), d['pipeline']['stage_ms'])"
done
