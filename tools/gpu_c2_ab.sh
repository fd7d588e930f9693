# Same-box sweep of one env knob on the config-2 line: rate and the one-stream stage times.
#   tools/gpu_c2_ab.sh VAR v1 v2 ...
set -o pipefail
V=$1; shift
mkdir -p gpurun_out
for x in "$@"; do
  env $V=$x timeout -k 10 200 python bench.py --cpu-sample 0 --no-e2e --sustain-repeats 0 --no-adversarial --no-config4 --no-wal > gpurun_out/c2ab_$x.json 2> gpurun_out/c2ab_$x.err || exit 1
  python -c "
import json; d=json.load(open('gpurun_out/c2ab_$x.json')); st=d['roofline']['stage_ms_one_stream']
print('$V=$x', d['correct'], round(d['value']/1e6,1), 'reduce', st.get('reduce'), 'final', st.get('final'))"
done
