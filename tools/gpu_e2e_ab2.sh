#!/bin/bash
# Pinned-input signature verify: first-batch share x steady chunk size, 3 interleaved repetitions.
set -o pipefail
mkdir -p gpurun_out/e2e2
for rep in 1 2 3; do
  for f in 0.5 0.62 0.7 0.78; do
    for cl in 17 18; do
      MV_STREAM_FIRST=$f MV_STREAM_CHUNK_LOG2=$cl timeout -k 10 120 python tools/pipe_probe.py > gpurun_out/e2e2/${f}_${cl}_$rep.log 2>&1 || { tail -5 gpurun_out/e2e2/${f}_${cl}_$rep.log; exit 1; }
      echo "rep=$rep first=$f chunk_log2=$cl $(grep pinned gpurun_out/e2e2/${f}_${cl}_$rep.log | sed 's/.*-> //')"
    done
  done
done
