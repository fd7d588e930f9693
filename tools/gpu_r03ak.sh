#!/bin/bash
# batch.hip compiled with the max-ilp machine scheduler (variant build, MV_LIB) vs the product:
# config-2 line, 2 interleaved reps.
set -o pipefail
mkdir -p gpurun_out/ilp
for rep in 1 2; do
for V in 0 ilp; do
  if [ $V = 0 ]; then L=""; else L="$GRAFT_REPO_ROOT/mysticeti_amd/_build/$V/libmysti_verify.so"; fi
  MV_LIB=$L timeout -k 10 300 python bench.py --steps 600 --warmup 10 --cpu-sample 0 --sustain-repeats 0 --no-adversarial --no-config4 --no-wal --no-config5 --no-e2e > gpurun_out/ilp/${V}_$rep.json 2> gpurun_out/ilp/${V}_$rep.err || { tail -5 gpurun_out/ilp/${V}_$rep.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/ilp/${V}_$rep.json')); print('rep $rep variant=$V', round(d['value']/1e6,1), d['correct'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
done
done
