#!/bin/bash
# A/B timing of experiment builds: tools/ab.sh [--path P] variant1 variant2 ...  ("main" = product lib)
set -o pipefail
mkdir -p gpurun_out
PATHARG="--path batch"
if [ "$1" = "--path" ]; then PATHARG="--path $2"; shift 2; fi
for v in "$@"; do
  if [ "$v" = main ]; then L=mysticeti_amd/libmysti_verify.so; else L=mysticeti_amd/_build/$v/libmysti_verify.so; fi
  MV_LIB=$PWD/$L timeout -k 10 120 python bench.py --steps 30 --warmup 3 --cpu-sample 0 --no-e2e $PATHARG > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || { tail -5 gpurun_out/ab_$v.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/ab_$v.json')); r=d['roofline']; print('$v', '$PATHARG', '|', round(d['value']/1e6,2), 'M/s', r['kernel'], r['kernel_ms'], d['correct'], (d['pipeline'].get('stage_ms') or {}))"
done
