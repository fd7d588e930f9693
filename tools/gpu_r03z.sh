#!/bin/bash
# Lane-per-string BLAKE2b variants (MV_B2_VAR: bit 0 prefetch, bit 1 rotl1 form, bit 2 five
# waves per SIMD): config 4 on one stream (stage hash ms) and as run, 2 interleaved reps.
set -o pipefail
mkdir -p gpurun_out/b2var
for rep in 1 2; do
for V in ${VS:-0 1 2 3 4 6}; do
  o=gpurun_out/b2var/c4_V${V}_$rep
  MV_B2_VAR=$V timeout -k 10 300 python bench.py --workload config4 --steps 20 --warmup 3 --cpu-sample 0 --host-fed-blocks 0 > $o.json 2> $o.err || { tail -5 $o.err; exit 1; }
  python3 -c "import json; d=json.load(open('$o.json')); p=d['pipeline']; print('rep $rep var=$V', round(d['value']/1e6,2), d['correct'], 'hash 1-stream', p['stage_ms']['hash'], 'as run', p['stage_ms_as_run']['hash'])"
done
done
