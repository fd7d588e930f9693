#!/bin/bash
# k_wal_crc rows in flight per wave (MV_WAL_ROWS 8 = product, 12 / 16 = variant builds loaded
# with MV_LIB): the WAL workload, 2 interleaved reps.
set -o pipefail
mkdir -p gpurun_out/walrows
for rep in 1 2; do
for V in ${VS:-0}; do
  if [ $V = 0 ]; then L=""; else L="$GRAFT_REPO_ROOT/mysticeti_amd/_build/$V/libmysti_verify.so"; fi
  MV_LIB=$L timeout -k 10 300 python bench.py --workload wal --steps 20 --warmup 3 --cpu-sample 0 > gpurun_out/walrows/r${V}_$rep.json 2> gpurun_out/walrows/r${V}_$rep.err || { tail -5 gpurun_out/walrows/r${V}_$rep.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/walrows/r${V}_$rep.json')); print('rep $rep variant=$V', d['value'], d['correct'], d['stage_ms'])"
done
done
