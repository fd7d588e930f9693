# Iteration check on the GPU box: batch-path GPU tests, a short config-2 line (stage times
# on one stream), the pinned-input end-to-end probe.   tools/gpu_iter.sh <tag> [pytest files]
set -o pipefail
TAG=${1:-it}; SEL=${2:-tests/test_gpu_batch.py}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest $SEL -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_$TAG.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED|Error" gpurun_out/pytest_$TAG.log | head -30; exit $rc; }
timeout -k 10 200 python bench.py --cpu-sample 0 --no-e2e --sustain-repeats 0 --no-adversarial --no-config4 > gpurun_out/${TAG}_c2.json 2> gpurun_out/${TAG}_c2.err || exit 1
python - <<PY
import json
d=json.load(open("gpurun_out/${TAG}_c2.json")); r=d["roofline"]
print("c2", round(d["value"]/1e6,1), "M/s", d["correct"], r["stage_ms_one_stream"])
PY
timeout -k 10 120 python tools/pipe_probe.py 2>&1 | grep -v H2D
