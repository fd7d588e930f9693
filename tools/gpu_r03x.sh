#!/bin/bash
# Submission queue A/B: linger / caller spin / pass-owner spin combos "L:QS:PS" (MV_Q_LINGER_US,
# MV_Q_SPIN_US, MV_PASS_SPIN), config-5 line per combo, REPS interleaved reps.
set -o pipefail
TAG=${1:-r03x}
mkdir -p gpurun_out/queue
if [ -z "$SKIPTEST" ]; then
  MV_Q_LINGER_US=50 MV_Q_SPIN_US=200 timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_blocks.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
  rc=$?; tail -2 gpurun_out/pytest_$TAG.log
  [ $rc -ne 0 ] && { grep -E "^E |FAILED" gpurun_out/pytest_$TAG.log | head -30; exit $rc; }
fi
for rep in $(seq 1 ${REPS:-2}); do
for C in ${CS:-0:0:0 50:0:0 50:0:1 50:200:0 50:200:1}; do
  IFS=: read L QS PS <<< "$C"
  o=gpurun_out/queue/${L}_${QS}_${PS}_$rep
  MV_Q_LINGER_US=$L MV_Q_SPIN_US=$QS MV_PASS_SPIN=$PS timeout -k 10 200 python bench.py --workload config5 --cpu-sample 0 --batches 1000 --conc-seconds 2 > $o.json 2> $o.err || { tail -5 $o.err; exit 1; }
  python - <<PY
import json
d=json.load(open("$o.json"))
v=d["shapes"]["config1"]; c=v["concurrent_1_block_callers"]["gpu"]; w=d["shapes"]["config4"]; c4=w["concurrent_1_block_callers"]["gpu"]
print("rep $rep $C c1 64-blk p50", v["gpu"]["p50_us"], "| c1 conc", c["blocks_per_s"], c["p50_us"], c["p99_us"], c["calls_per_device_pass"], "| c4 conc", c4["blocks_per_s"], c4["p50_us"], c4["calls_per_device_pass"])
PY
done
done
