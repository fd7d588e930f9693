#!/bin/bash
# Zero-copy pinned signature verify: batch tests, then pinned end-to-end zero-copy vs chunked copy
# (3 interleaved repetitions) and the first-batch share of the zero-copy path.
set -o pipefail
TAG=${1:-r03t}
mkdir -p gpurun_out/zc
timeout -k 10 400 python -u -m pytest tests/test_gpu_batch.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_$TAG.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED" gpurun_out/pytest_$TAG.log | head -30; exit $rc; }
for rep in 1 2 3; do
  for cfg in "0 0.5" "1 0.5" "1 0.6" "1 0.7"; do
    set -- $cfg
    MV_SIG_ZEROCOPY=$1 MV_ZC_FIRST=$2 MV_STREAM_FIRST=0.7 timeout -k 10 120 python tools/pipe_probe.py > gpurun_out/zc/${1}_${2}_$rep.log 2>&1 || { tail -5 gpurun_out/zc/${1}_${2}_$rep.log; exit 1; }
    echo "rep=$rep zerocopy=$1 first=$2 $(grep pinned gpurun_out/zc/${1}_${2}_$rep.log | sed 's/.*-> //')"
  done
done
