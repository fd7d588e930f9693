#!/bin/bash
# Pinned end-to-end signature verify: kernel + memory-copy timeline of the last of three calls.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/e2etl
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/e2etl/tr -o run -f csv -- python tools/e2e_probe.py > gpurun_out/e2etl/probe.log 2>&1
rc=$?; cat gpurun_out/e2etl/probe.log | grep call
python tools/timeline.py gpurun_out/e2etl/tr 7 > gpurun_out/e2etl/timeline.txt; wc -l gpurun_out/e2etl/timeline.txt
exit $rc
