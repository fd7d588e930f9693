#!/bin/bash
# Linger target share A/B (MV_Q_LINGER_PCT 100 / 75 / 50) at linger 50 us, config-5 line, 3 reps.
set -o pipefail
mkdir -p gpurun_out/lpct
for rep in 1 2 3; do
for P in 100 75 50; do
  o=gpurun_out/lpct/P${P}_$rep
  MV_Q_LINGER_PCT=$P timeout -k 10 200 python bench.py --workload config5 --cpu-sample 0 --batches 500 --conc-seconds 2 > $o.json 2> $o.err || { tail -5 $o.err; exit 1; }
  python - <<PY
import json
d=json.load(open("$o.json"))
v=d["shapes"]["config1"]; c=v["concurrent_1_block_callers"]["gpu"]; w=d["shapes"]["config4"]; c4=w["concurrent_1_block_callers"]["gpu"]
print("rep $rep pct=$P c1 conc", c["blocks_per_s"], c["p50_us"], c["p99_us"], c["calls_per_device_pass"], "| c4 conc", c4["blocks_per_s"], c4["p50_us"], c4["calls_per_device_pass"])
PY
done
done
