#!/bin/bash
# Pass-set-owned scratch: block tests; config-5 line and host pass cost, two-kernel vs fused ingest+hash.
set -o pipefail
TAG=${1:-r03o}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_blocks.py tests/test_gpu_engine.py tests/test_gpu_ingest.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_$TAG.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED" gpurun_out/pytest_$TAG.log | head -30; exit $rc; }
for f in 0 1; do
  MV_BLK_FUSED=$f timeout -k 10 200 python bench.py --workload config5 --cpu-sample 0 --batches 2000 --conc-seconds 2 > gpurun_out/c5_f${f}_$TAG.json 2> gpurun_out/c5_f${f}_$TAG.err || { tail -5 gpurun_out/c5_f${f}_$TAG.err; exit 1; }
  MV_BLK_FUSED=$f MV_BLK_TRACE=1 timeout -k 10 200 python bench.py --workload config5 --cpu-sample 0 --batches 300 --conc-seconds 0.5 > /dev/null 2> gpurun_out/c5_tr${f}_$TAG.err || { tail -5 gpurun_out/c5_tr${f}_$TAG.err; exit 1; }
  python - <<PY
import json, re, statistics as S
d=json.load(open("gpurun_out/c5_f${f}_$TAG.json"))
v=d["shapes"]["config1"]; c=v["concurrent_1_block_callers"]["gpu"]; w=d["shapes"]["config4"]
rows=[l for l in open("gpurun_out/c5_tr${f}_$TAG.err") if "[blk]" in l][-400:]
k=[float(re.search(r'kernels ([0-9.]+)', l).group(1)) for l in rows]
print("fused=$f c1 64-blk p50", v["gpu"]["p50_us"], v["gpu"]["p99_us"], "conc", c["blocks_per_s"], c["p50_us"], "| c4 64-blk", w["gpu"]["p50_us"], "| enqueue us median", S.median(k))
PY
done
