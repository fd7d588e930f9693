#!/bin/bash
# Segmented WAL check (walk segments on a second stream beside the crc of the walked ones):
# WAL tests, then the WAL workload with MV_WAL_PIPE 1 / 0, 2 interleaved reps.
set -o pipefail
TAG=${1:-r03ai}
mkdir -p gpurun_out/walpipe
timeout -k 10 400 python -u -m pytest tests/test_wal.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_$TAG.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED" gpurun_out/pytest_$TAG.log | head -30; exit $rc; }
for rep in 1 2; do
for P in ${PS:-1 0}; do
  MV_WAL_PIPE=${P%:*} MV_WAL_SEGS=${P#*:} timeout -k 10 300 python bench.py --workload wal --steps 20 --warmup 3 --cpu-sample 0 > gpurun_out/walpipe/p${P/:/_}_$rep.json 2> gpurun_out/walpipe/p${P/:/_}_$rep.err || { tail -5 gpurun_out/walpipe/p${P/:/_}_$rep.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/walpipe/p${P/:/_}_$rep.json')); print('rep $rep pipe=$P', d['value'], d['correct'], d['ms_per_step'], d['stage_ms'])"
done
done
