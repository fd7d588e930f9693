#!/bin/bash
# Run-ahead WAL walk: WAL tests, then the WAL workload (2 reps) with its kernel trace.
set -o pipefail
TAG=${1:-r03ag}
mkdir -p gpurun_out/walk
timeout -k 10 400 python -u -m pytest tests/test_wal.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_$TAG.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED" gpurun_out/pytest_$TAG.log | head -30; exit $rc; }
for rep in 1 2; do
  timeout -k 10 300 python bench.py --workload wal --steps 20 --warmup 3 --cpu-sample 0 > gpurun_out/walk/wal_$rep.json 2> gpurun_out/walk/wal_$rep.err || { tail -5 gpurun_out/walk/wal_$rep.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/walk/wal_$rep.json')); print('rep $rep', d['value'], d.get('unit'), d.get('correct'), d.get('ms_per_step'), d.get('stage_ms', d.get('pipeline')))"
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/walk/tr -o run -- python bench.py --workload wal --steps 5 --warmup 1 --cpu-sample 0 > gpurun_out/walk/tr.log 2>&1 || { tail -5 gpurun_out/walk/tr.log; exit 1; }
python3 - <<PY
import csv
for r in csv.DictReader(open("gpurun_out/walk/tr/run_kernel_stats.csv")):
    print(r["Name"][:50], r["Calls"], round(float(r["AverageNs"])/1e3,1), "us")
PY
