#!/bin/bash
# Session-3 GPU call: GPU tests, the default bench line, then stream-count A/B for configs 2 and 4
# and the config-5 latency line.
set -o pipefail
TAG=${1:-s3}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu_$TAG.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED" gpurun_out/pytest_gpu_$TAG.log | head -30; exit $rc; }
timeout -k 10 300 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit 1
for S in 2 3; do
  timeout -k 10 200 python bench.py --streams $S --cpu-sample 0 --no-e2e --sustain-repeats 1 --no-adversarial --no-config4 --no-wal > gpurun_out/${TAG}_c2_s$S.json 2> gpurun_out/${TAG}_c2_s$S.err || exit 1
  timeout -k 10 300 python bench.py --workload config4 --streams $S --cpu-sample 0 > gpurun_out/${TAG}_c4_s$S.json 2> gpurun_out/${TAG}_c4_s$S.err || exit 1
done
timeout -k 10 300 python bench.py --workload config5 > gpurun_out/${TAG}_c5.json 2> gpurun_out/${TAG}_c5.err || exit 1
python - <<PY
import json
for S in (2, 3):
    d=json.load(open(f"gpurun_out/${TAG}_c2_s{S}.json"))
    print("c2 streams", S, round(d["value"]/1e6,1), "M/s", d["correct"], (d.get("sustained") or {}).get("median"))
    d=json.load(open(f"gpurun_out/${TAG}_c4_s{S}.json")); d=d.get("config4") or d
    print("c4 streams", S, round(d["value"]/1e6,1), "M/s", d["correct"])
d=json.load(open("gpurun_out/bench_${TAG}.json"))
print("default", d["value"], d["roofline"]["frac"], d["end_to_end"], (d.get("config4") or {}).get("value"))
PY
