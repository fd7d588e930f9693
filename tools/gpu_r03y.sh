#!/bin/bash
# Lane-per-string BLAKE2b (blake2b_lane.hip) vs the quad kernel with plain 64-bit adds: hash /
# block / ingest tests, then config 4 with MV_B2_LANE 1 / 0 (2 interleaved reps) and a
# 1-stream kernel trace of each.
set -o pipefail
TAG=${1:-r03y}
mkdir -p gpurun_out/b2lane
timeout -k 10 500 python -u -m pytest tests/test_gpu_primitives.py tests/test_gpu_blocks.py tests/test_gpu_ingest.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_$TAG.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED" gpurun_out/pytest_$TAG.log | head -30; exit $rc; }
for rep in 1 2; do
for L in 1 0; do
  o=gpurun_out/b2lane/c4_L${L}_$rep
  MV_B2_LANE=$L timeout -k 10 300 python bench.py --workload config4 --steps 20 --warmup 3 --cpu-sample 0 --host-fed-blocks 0 > $o.json 2> $o.err || { tail -5 $o.err; exit 1; }
  python3 -c "import json; d=json.load(open('$o.json')); p=d['pipeline']; print('rep $rep lane=$L', round(d['value']/1e6,2), d['correct'], 'as_run', p['stage_ms_as_run'], '1stream', p['stage_ms'])"
done
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for L in 1 0; do
  MV_B2_LANE=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/b2lane/tr$L -o run -- python bench.py --workload config4 --steps 3 --warmup 1 --cpu-sample 0 --streams 1 --host-fed-blocks 0 > gpurun_out/b2lane/tr$L.log 2>&1 || { tail -5 gpurun_out/b2lane/tr$L.log; exit 1; }
  grep -E "k_b2|k_block_ingest" gpurun_out/b2lane/tr$L/run_kernel_stats.csv | cut -d, -f1-4 | cut -c1-40,200-
done
