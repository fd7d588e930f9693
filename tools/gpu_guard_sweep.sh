# Guarded sub-batch count sweep: the adversarial leg of config 2 at MV_GUARD_GROUPS = 4, 8, 16.
#   tools/gpu_guard_sweep.sh
set -o pipefail
mkdir -p gpurun_out
for g in 4 8 16; do
  MV_GUARD_GROUPS=$g timeout -k 10 200 python bench.py --cpu-sample 0 --no-e2e --sustain-repeats 0 --no-config4 --no-wal --steps 200 > gpurun_out/guard_$g.json 2> gpurun_out/guard_$g.err || exit 1
  python -c "
import json; d=json.load(open('gpurun_out/guard_$g.json')); a=d['adversarial']
print($g, round(d['value']/1e6,1), {k:(round(v['value']/1e6,1), v['ratio_to_all_valid'], v['correct']) for k,v in a.items() if isinstance(v,dict)})"
done
