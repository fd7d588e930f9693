#!/bin/bash
# Streamed pinned verify with signature copies on a second copy stream (MV_STREAM_COPY2 1 / 0):
# batch tests, then the pinned end-to-end probe (3 interleaved reps) and the config-2 line.
set -o pipefail
TAG=${1:-r03af}
mkdir -p gpurun_out/copy2
timeout -k 10 400 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_$TAG.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED" gpurun_out/pytest_$TAG.log | head -30; exit $rc; }
for rep in 1 2 3; do
for C in 1 0; do
  MV_STREAM_COPY2=$C timeout -k 10 120 python tools/e2e_probe.py > gpurun_out/copy2/p${C}_$rep.log 2>&1 || { tail -5 gpurun_out/copy2/p${C}_$rep.log; exit 1; }
  echo "rep $rep copy2=$C $(grep 'call 2' gpurun_out/copy2/p${C}_$rep.log)"
done
done
for C in 1 0; do
  MV_STREAM_COPY2=$C timeout -k 10 300 python bench.py --steps 300 --warmup 5 --cpu-sample 0 --sustain-repeats 0 --no-adversarial --no-config4 --no-wal --no-config5 > gpurun_out/copy2/c2_$C.json 2> gpurun_out/copy2/c2_$C.err || { tail -5 gpurun_out/copy2/c2_$C.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/copy2/c2_$C.json')); print('copy2=$C c2', round(d['value']/1e6,1), 'e2e', round(d['end_to_end']['value']/1e6,1), 'pageable', round(d['end_to_end']['pageable']/1e6,1))"
done
