#!/bin/bash
# Full GPU test suite, then the round-3 rocprof traces + PMC passes (tools/profile_r03.sh).
set -o pipefail
TAG=${1:-r03aa}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_$TAG.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED" gpurun_out/pytest_$TAG.log | head -30; exit $rc; }
bash tools/profile_r03.sh
