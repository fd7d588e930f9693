#!/bin/bash
# Pinned-input signature verify (PCIe-inclusive): batches per call x copy-chunk size A/B.
#   tools/gpu_e2e_ab.sh <tag>
set -o pipefail
TAG=${1:-e2e}
mkdir -p gpurun_out
for nb in 1 2; do
  for cl in 17 18; do
    MV_STREAM_BATCHES=$nb MV_STREAM_CHUNK_LOG2=$cl timeout -k 10 120 python tools/pipe_probe.py > gpurun_out/e2e_${nb}_${cl}_$TAG.log 2>&1 || { tail -5 gpurun_out/e2e_${nb}_${cl}_$TAG.log; exit 1; }
    echo "batches=$nb chunk_log2=$cl: $(grep pinned gpurun_out/e2e_${nb}_${cl}_$TAG.log)"
  done
done
