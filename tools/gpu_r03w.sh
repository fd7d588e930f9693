#!/bin/bash
# Submission-queue linger A/B (MV_Q_LINGER_US 0 / 10 / 25 / 50): engine tests with linger on,
# then the config-5 line per setting, 2 interleaved reps.
set -o pipefail
TAG=${1:-r03w}
mkdir -p gpurun_out/linger
[ -n "$SKIPTEST" ] || MV_Q_LINGER_US=25 timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_blocks.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_$TAG.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED" gpurun_out/pytest_$TAG.log | head -30; exit $rc; }
for rep in 1 2; do
for L in ${LS:-0 10 25 50}; do
  o=gpurun_out/linger/L${L}_$rep
  MV_Q_LINGER_US=${L%s} MV_PASS_SPIN=$([ "${L%s}" != "$L" ] && echo 1 || echo 0) timeout -k 10 200 python bench.py --workload config5 --cpu-sample 0 --batches 1000 --conc-seconds 2 > $o.json 2> $o.err || { tail -5 $o.err; exit 1; }
  python - <<PY
import json
d=json.load(open("$o.json"))
v=d["shapes"]["config1"]; c=v["concurrent_1_block_callers"]["gpu"]; w=d["shapes"]["config4"]; c4=w["concurrent_1_block_callers"]["gpu"]
print("rep $rep linger=$L c1 64-blk p50", v["gpu"]["p50_us"], "| c1 conc", c["blocks_per_s"], c["p50_us"], c["p99_us"], c["calls_per_device_pass"], "| c4 conc", c4["blocks_per_s"], c4["p50_us"], c4["calls_per_device_pass"])
PY
done
done
