#!/bin/bash
# Row-form field ops (fe_r16.h) and k_verify_comb16: chain microbench, primitive / comb / block
# GPU tests, config-5 latency; host-fed config 4 with 8 vs 16 pack threads.
#   tools/gpu_r03e.sh <tag>
set -o pipefail
TAG=${1:-r03e}
mkdir -p gpurun_out
timeout -k 10 60 tools/microbench_chain > gpurun_out/chain_$TAG.jsonl 2>&1 || { cat gpurun_out/chain_$TAG.jsonl; exit 1; }
cat gpurun_out/chain_$TAG.jsonl
timeout -k 10 400 python -u -m pytest tests/test_gpu_primitives.py tests/test_gpu_comb.py tests/test_gpu_blocks.py tests/test_gpu_engine.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_$TAG.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED|Error" gpurun_out/pytest_$TAG.log | head -30; exit $rc; }
timeout -k 10 200 python bench.py --workload config5 --cpu-sample 0 --batches 2000 --conc-seconds 1 > gpurun_out/c5_$TAG.json 2> gpurun_out/c5_$TAG.err || { tail -5 gpurun_out/c5_$TAG.err; exit 1; }
python - <<PY
import json
d=json.load(open("gpurun_out/c5_$TAG.json"))
for s,v in d["shapes"].items():
    c=v["concurrent_1_block_callers"]["gpu"]
    print(s, v["gpu"]["p50_us"], v["gpu"]["p99_us"], "conc", c["blocks_per_s"], c["p50_us"], c["calls_per_device_pass"])
PY
for th in 8 16; do
  MV_PACK_THREADS=$th timeout -k 10 300 python bench.py --workload config4 --batch 262144 --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/c4hf_${th}_$TAG.json 2> gpurun_out/c4hf_${th}_$TAG.err || { tail -5 gpurun_out/c4hf_${th}_$TAG.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/c4hf_${th}_$TAG.json')); h=d['host_fed']; print('pack threads $th', h['value'], h['frac_of_pcie_bound'], h['h2d_GBps_pinned'])"
done
