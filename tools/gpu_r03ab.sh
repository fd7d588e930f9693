#!/bin/bash
# Block calls of batch size in two halves (second half's parse beside the first half's hash on
# another stream, MV_BLK_PIPE): block / ingest / engine tests, then config 4 with MV_BLK_PIPE
# 1 / 0 at 2 and 1 bench streams, 2 interleaved reps.
set -o pipefail
TAG=${1:-r03ab}
mkdir -p gpurun_out/pipe
timeout -k 10 500 python -u -m pytest tests/test_gpu_blocks.py tests/test_gpu_ingest.py tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_$TAG.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED" gpurun_out/pytest_$TAG.log | head -30; exit $rc; }
for rep in 1 2; do
for C in 1:2 0:2 1:1 0:1; do
  IFS=: read P S <<< "$C"
  o=gpurun_out/pipe/c4_P${P}_S${S}_$rep
  MV_BLK_PIPE=$P timeout -k 10 300 python bench.py --workload config4 --steps 20 --warmup 3 --cpu-sample 0 --host-fed-blocks 0 --streams $S > $o.json 2> $o.err || { tail -5 $o.err; exit 1; }
  python3 -c "import json; d=json.load(open('$o.json')); p=d['pipeline']; print('rep $rep pipe=$P streams=$S', round(d['value']/1e6,2), d['correct'], d['ms_per_step'])"
done
done
