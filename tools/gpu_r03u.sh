#!/bin/bash
# Config 4: ingest occupancy cap by LDS padding (0 / 6 KB / 12 KB / 22 KB per workgroup), 2 reps.
set -o pipefail
mkdir -p gpurun_out/c4pad
for rep in 1 2; do
  for pad in 0 6144 12288 22528; do
    MV_INGEST_LDS_PAD=$pad timeout -k 10 300 python bench.py --workload config4 --steps 20 --warmup 3 --cpu-sample 0 --host-fed-blocks 0 > gpurun_out/c4pad/${pad}_$rep.json 2> gpurun_out/c4pad/${pad}_$rep.err || { tail -5 gpurun_out/c4pad/${pad}_$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/c4pad/${pad}_$rep.json')); print('rep $rep pad $pad', round(d['value']/1e6,2), d['correct'], d['pipeline']['stage_ms_as_run']['parse'], d['pipeline']['stage_ms_as_run']['hash'])"
  done
done
