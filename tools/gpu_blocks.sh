#!/bin/bash
# GPU check of the block paths: parity tests (new + existing), then the config-5 and config-4
# bench lines and the default config-2 line.
#   tools/gpu_blocks.sh <tag>
set -o pipefail
TAG=${1:-blk}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_$TAG.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED|Error" gpurun_out/pytest_$TAG.log | head -40; exit $rc; }
timeout -k 10 300 python bench.py --workload config5 --batches ${C5_BATCHES:-10000} \
  > gpurun_out/c5_$TAG.json 2> gpurun_out/c5_$TAG.err || { tail -20 gpurun_out/c5_$TAG.err; exit 1; }
cat gpurun_out/c5_$TAG.json
timeout -k 10 400 python bench.py --workload config4 --batch ${C4_BATCH:-1048576} --steps ${C4_STEPS:-10} --warmup 2 \
  > gpurun_out/c4_$TAG.json 2> gpurun_out/c4_$TAG.err || { tail -20 gpurun_out/c4_$TAG.err; exit 1; }
cat gpurun_out/c4_$TAG.json
[ "${NOC2:-0}" = 1 ] && exit 0
timeout -k 10 300 python bench.py > gpurun_out/c2_$TAG.json 2> gpurun_out/c2_$TAG.err || { tail -20 gpurun_out/c2_$TAG.err; exit 1; }
cat gpurun_out/c2_$TAG.json
