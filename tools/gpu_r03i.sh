#!/bin/bash
# k_bv_bucket with V in LDS: batch GPU tests, config-2 line (stage times), e2e with 3 / 4
# batches per call.   tools/gpu_r03i.sh <tag>
set -o pipefail
TAG=${1:-r03i}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_verify.py tests/test_gpu_primitives.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_$TAG.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED" gpurun_out/pytest_$TAG.log | head -30; exit $rc; }
timeout -k 10 300 python bench.py --cpu-sample 0 --no-config5 --no-wal --no-adversarial --no-config4 --sustain-repeats 3 > gpurun_out/c2_$TAG.json 2> gpurun_out/c2_$TAG.err || { tail -5 gpurun_out/c2_$TAG.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/c2_$TAG.json')); print('c2', round(d['value']/1e6,1), d['correct'], 'sust', d['sustained']['median'], 'frac', d['roofline']['frac'], d['roofline']['stage_ms_one_stream']); print('e2e', d['end_to_end']['value'])"
for nb in 3 4; do
  MV_STREAM_BATCHES=$nb timeout -k 10 120 python tools/pipe_probe.py > gpurun_out/e2e_${nb}_$TAG.log 2>&1 || { tail -5 gpurun_out/e2e_${nb}_$TAG.log; exit 1; }
  echo "batches=$nb: $(grep pinned gpurun_out/e2e_${nb}_$TAG.log)"
done
