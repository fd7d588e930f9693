#!/bin/bash
# Field-op chain latency microbench, PMC passes on the fused ingest+hash kernel, config-5
# latency with the fused and the two-kernel block path.
#   tools/gpu_r03c.sh <tag>
set -o pipefail
TAG=${1:-r03c}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 60 tools/microbench_chain > gpurun_out/chain_$TAG.jsonl 2>&1 || { cat gpurun_out/chain_$TAG.jsonl; exit 1; }
cat gpurun_out/chain_$TAG.jsonl
timeout -k 10 400 bash tools/pmc_ingest.sh ih_$TAG k_block_ingest_hash > gpurun_out/pmc_ih_$TAG.txt 2>&1 || { tail -20 gpurun_out/pmc_ih_$TAG.txt; exit 1; }
tail -30 gpurun_out/pmc_ih_$TAG.txt
for k in fused old; do
  if [ $k = old ]; then export MV_BLK_FUSED=0; else unset MV_BLK_FUSED; fi
  timeout -k 10 200 python bench.py --workload config5 --cpu-sample 0 --batches 2000 --conc-seconds 1 > gpurun_out/c5_${k}_$TAG.json 2> gpurun_out/c5_${k}_$TAG.err || { tail -5 gpurun_out/c5_${k}_$TAG.err; exit 1; }
done
python - <<PY
import json
for k in ("fused","old"):
    d=json.load(open(f"gpurun_out/c5_{k}_$TAG.json"))
    for s,v in d["shapes"].items():
        c=v["concurrent_1_block_callers"]["gpu"]
        print(k, s, v["gpu"]["p50_us"], v["gpu"]["p99_us"], "conc", c["blocks_per_s"], c["p50_us"])
PY
