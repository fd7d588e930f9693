#!/bin/bash
# One GPU call: parity tests, the default bench line (with CPU baseline), rocprof evidence.
#   tools/round_gpu.sh <tag>
set -o pipefail
TAG=${1:-r01}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_gpu_$TAG.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED" gpurun_out/pytest_gpu_$TAG.log | head -30; exit $rc; }
timeout -k 10 300 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit 1
cat gpurun_out/bench_$TAG.json
[ "${NOPROF:-0}" = 1 ] && exit 0
bash tools/profile.sh $TAG
