#!/bin/bash
# WAL row (f4): GPU tests, then the WAL bench line
set -o pipefail
TAG=${1:-wal}; N=${2:-1048576}
mkdir -p gpurun_out/$TAG
timeout -k 10 300 python -u -m pytest tests/test_wal.py tests/test_abi.py -x -v --timeout 120 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1
rc=$?; tail -14 gpurun_out/$TAG/pytest.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED|Error" gpurun_out/$TAG/pytest.log | head -30; exit $rc; }
timeout -k 10 300 python bench.py --workload wal --wal-entries $N --steps 10 --warmup 2 > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || { tail -20 gpurun_out/$TAG/bench.err; exit 1; }
cat gpurun_out/$TAG/bench.json
