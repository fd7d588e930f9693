#!/bin/bash
# Round-3 final evidence, part A: every GPU test, smoke, the default bench line (the driver's
# shape), the --gpus 2 self-launch rehearsal.   tools/final_r03.sh -> gpurun_out/final_r03/
set -o pipefail
OUT=gpurun_out/final_r03
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -2 $OUT/pytest_gpu.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED" $OUT/pytest_gpu.log | head -30; exit $rc; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail -5 $OUT/bench_default.err; exit 1; }
echo "default line done"
timeout -k 10 400 python bench.py --gpus 2 --steps 200 --warmup 5 --no-e2e --sustain-repeats 1 --no-config5 --no-wal --host-fed-blocks 0 --cpu-sample 0 > $OUT/bench_gpus2.json 2> $OUT/bench_gpus2.err || { tail -5 $OUT/bench_gpus2.err; exit 1; }
python - <<PY
import json
d=json.load(open("$OUT/bench_default.json"))
print("c2", round(d["value"]/1e6,1), d["correct"], "frac", d["roofline"]["frac"], "sust", round(d["sustained"]["median"]/1e6,1))
c4=d["config4"]; print("c4", round(c4["value"]/1e6,1), "host_fed", c4["host_fed"]["value"], c4["host_fed"]["pageable"], "e2e", round(d["end_to_end"]["value"]/1e6,1), "wal", d["wal"]["value"])
for s,v in d["config5"]["shapes"].items():
    c=v["concurrent_1_block_callers"]
    print("c5", s, "gpu", v["gpu"]["p50_us"], v["gpu"]["p99_us"], "cpu16", v.get("cpu_16t",{}).get("p50_us"), "conc gpu", c["gpu"]["blocks_per_s"], "cpu", c.get("cpu_own_core",{}).get("blocks_per_s"))
d2=json.load(open("$OUT/bench_gpus2.json")); print("gpus2", d2["n_gpus"], round(d2["value"]/1e6,1), d2["correct"])
PY
