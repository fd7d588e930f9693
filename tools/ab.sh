#!/bin/bash
# A/B timing of experiment builds: tools/ab.sh variant1 variant2 ...  ("main" = product lib)
set -o pipefail
mkdir -p gpurun_out
for v in "$@"; do
  if [ "$v" = main ]; then L=mysticeti_amd/libmysti_verify.so; else L=mysticeti_amd/_build/$v/libmysti_verify.so; fi
  MV_LIB=$PWD/$L timeout -k 10 120 python bench.py --steps 10 --warmup 2 --cpu-sample 0 --no-e2e > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || { tail -5 gpurun_out/ab_$v.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/ab_$v.json')); print('$v', d['value'], d['roofline']['kernel_ms'], d['correct'], d['parity_sha256'])"
done
