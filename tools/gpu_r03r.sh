#!/bin/bash
# Host-fed config 4: kernel + memory-copy timeline of the host-fed leg (the last ~90 ms of the run).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/hftl -o run -f csv -- python bench.py --workload config4 --batch 65536 --steps 2 --warmup 1 --cpu-sample 0 > gpurun_out/hftl.log 2>&1 || { tail -5 gpurun_out/hftl.log; exit 1; }
python tools/timeline.py gpurun_out/hftl 400 > gpurun_out/hf_timeline.txt
grep -c . gpurun_out/hf_timeline.txt
