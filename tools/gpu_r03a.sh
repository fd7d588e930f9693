#!/bin/bash
# Round-3 GPU check: GPU tests, smoke, the default bench line (driver shape), the --gpus 2
# self-launch rehearsal (both ranks on device 0).
#   tools/gpu_r03a.sh <tag> [skip_tests]
set -o pipefail
TAG=${1:-r03a}
mkdir -p gpurun_out
if [ -z "$2" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu_$TAG.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED" gpurun_out/pytest_gpu_$TAG.log | head -30; exit $rc; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { tail -5 gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
fi
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -5 gpurun_out/bench_$TAG.err; exit 1; }
echo "bench 1 done"
timeout -k 10 500 python bench.py --gpus 2 --steps 20 --warmup 5 --no-e2e --sustain-repeats 1 > gpurun_out/bench2_$TAG.json 2> gpurun_out/bench2_$TAG.err || { tail -5 gpurun_out/bench2_$TAG.err; exit 1; }
python - <<PY
import json
d=json.load(open("gpurun_out/bench_$TAG.json"))
print("c2", round(d["value"]/1e6,1), d["correct"], "frac", d["roofline"]["frac"], "sust", round(d["sustained"]["median"]/1e6,1))
print("c4", round(d["config4"]["value"]/1e6,1), "e2e", round(d["end_to_end"]["value"]/1e6,1), "wal", d["wal"]["value"])
for s,v in d["config5"]["shapes"].items():
    c=v["concurrent_1_block_callers"]
    print("c5", s, "gpu", v["gpu"]["p50_us"], v["gpu"]["p99_us"], "cpu1", v.get("cpu_1t",{}).get("p50_us"), "cpuN", [v[k]["p50_us"] for k in v if k.startswith("cpu_") and k!="cpu_1t" and isinstance(v[k],dict) and "p50_us" in v[k]],
          "conc gpu", c["gpu"]["blocks_per_s"], c["gpu"]["p50_us"], "cpu", c.get("cpu_own_core",{}).get("blocks_per_s"))
d2=json.load(open("gpurun_out/bench2_$TAG.json"))
print("gpus2 n_gpus", d2["n_gpus"], round(d2["value"]/1e6,1), d2["correct"])
PY
