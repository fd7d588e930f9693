#!/bin/bash
# Round-2 evidence on the committed tree: full GPU tests, default bench line, rocprof (tools/profile_r02.sh).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_r02p.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_r02p.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED|Error" gpurun_out/pytest_r02p.log | head -30; exit $rc; }
timeout -k 10 400 python bench.py > gpurun_out/bench_r02p.json 2> gpurun_out/bench_r02p.err || exit 1
cat gpurun_out/bench_r02p.json
bash tools/profile_r02.sh r02p
