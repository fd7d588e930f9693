set -o pipefail
timeout -k 10 200 python bench.py --cpu-sample 0 --sustain-repeats 0 --no-adversarial --no-config4 --no-wal > gpurun_out/b1.json 2> gpurun_out/b.err || exit 1
python -c "
import json; d=json.load(open('gpurun_out/b1.json')); print('short', round(d['value']/1e6,1), d['end_to_end']['value']/1e6, d['end_to_end']['pageable']/1e6)"
timeout -k 10 200 python bench.py --cpu-sample 0 --sustain-repeats 0 --no-adversarial --no-config4 --no-wal --streams 1 > gpurun_out/b2.json 2> gpurun_out/b.err || exit 1
python -c "
import json; d=json.load(open('gpurun_out/b2.json')); print('1stream', round(d['value']/1e6,1), d['end_to_end']['value']/1e6, d['end_to_end']['pageable']/1e6)"
timeout -k 10 120 python tools/pipe_probe.py 2>&1 | grep -v H2D || exit 1
