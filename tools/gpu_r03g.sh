#!/bin/bash
# Phase timing of the online comb verify, then the pinned-input signature streaming timeline.
#   tools/gpu_r03g.sh <tag>
set -o pipefail
TAG=${1:-r03g}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 60 tools/comb_phase > gpurun_out/comb_phase_$TAG.jsonl 2>&1 || { cat gpurun_out/comb_phase_$TAG.jsonl; exit 1; }
cat gpurun_out/comb_phase_$TAG.jsonl
timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/tl_$TAG -o run -f csv -- python tools/pipe_probe.py > gpurun_out/tl_$TAG.log 2>&1 || { tail -5 gpurun_out/tl_$TAG.log; exit 1; }
cat gpurun_out/tl_$TAG.log | grep -v "^W\|^\[" | tail -5
python tools/timeline.py gpurun_out/tl_$TAG 7 > gpurun_out/timeline_$TAG.txt
echo done
