#!/bin/bash
# Config 2: bench streams 2 / 3 / 4 (steps alternate over them), 2 interleaved reps.
set -o pipefail
mkdir -p gpurun_out/c2streams
for rep in 1 2; do
for S in 2 3 4; do
  timeout -k 10 300 python bench.py --steps 600 --warmup 10 --cpu-sample 0 --sustain-repeats 0 --no-adversarial --no-config4 --no-wal --no-config5 --no-e2e --streams $S > gpurun_out/c2streams/s${S}_$rep.json 2> gpurun_out/c2streams/s${S}_$rep.err || { tail -5 gpurun_out/c2streams/s${S}_$rep.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/c2streams/s${S}_$rep.json')); print('rep $rep streams=$S', round(d['value']/1e6,1), d['correct'], d['ms_per_step'])"
done
done
