#!/bin/bash
# Round-2 final GPU evidence: all GPU tests, smoke, the default bench line, the config-5 line.
#   tools/final_r02.sh <tag>
set -o pipefail
TAG=${1:-r02f}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu_$TAG.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED" gpurun_out/pytest_gpu_$TAG.log | head -30; exit $rc; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { tail -5 gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 400 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -5 gpurun_out/bench_$TAG.err; exit 1; }
timeout -k 10 300 python bench.py --workload config5 > gpurun_out/bench_c5_$TAG.json 2> gpurun_out/bench_c5_$TAG.err || { tail -5 gpurun_out/bench_c5_$TAG.err; exit 1; }
python - <<PY
import json
d=json.load(open("gpurun_out/bench_$TAG.json"))
print("c2", round(d["value"]/1e6,1), d["correct"], "frac", d["roofline"]["frac"], "sust", round(d["sustained"]["median"]/1e6,1))
print("adv", {k:(round(v["value"]/1e6,1), v["ratio_to_all_valid"]) for k,v in d["adversarial"].items() if isinstance(v,dict)})
print("c4", round(d["config4"]["value"]/1e6,1), "e2e", round(d["end_to_end"]["value"]/1e6,1), round(d["end_to_end"]["pageable"]/1e6,1), "wal", d["wal"]["value"])
c=json.load(open("gpurun_out/bench_c5_$TAG.json"))
for s,v in c["shapes"].items(): print("c5", s, v["gpu"]["p50_us"], v.get("cpu_16t",{}).get("p50_us"), v["concurrent_1_block_callers"]["gpu"]["p50_us"])
PY
