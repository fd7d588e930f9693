set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_verify.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_batch.log 2>&1 || { tail -30 gpurun_out/pt_batch.log; exit 1; }
tail -2 gpurun_out/pt_batch.log
timeout -k 10 120 python bench.py --steps 10 --warmup 2 --cpu-sample 0 --no-e2e --path batch > gpurun_out/b_batch.json 2> gpurun_out/b_batch.err || { tail gpurun_out/b_batch.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/b_batch.json')); print(d['value'], d['roofline']['kernel_ms'], d['correct'], d['parity_sha256'])"
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_batch -o run -- python bench.py --steps 5 --warmup 1 --cpu-sample 0 --no-e2e --path batch --streams 1 > gpurun_out/prof_batch.log 2>&1
python - <<'PY'
import csv
for r in csv.DictReader(open('gpurun_out/prof_batch/run_kernel_stats.csv')):
    print(r['Name'][:40], r['Calls'], round(float(r['AverageNs'])/1e3, 1), 'us')
PY
