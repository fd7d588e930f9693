set -o pipefail
timeout -k 10 300 python bench.py --workload config4 --cpu-sample 0 --batch 2097152 > gpurun_out/c4big.json 2> gpurun_out/c4big.err || { tail -5 gpurun_out/c4big.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/c4big.json')); d=d.get('config4') or d
print('c4 2^21', round(d['value']/1e6,1), d['correct'], d['pipeline']['stage_ms'])"
