# Same-box A/B of the config-5 latency line under an env toggle.   tools/gpu_c5_ab.sh VAR A B
set -o pipefail
V=$1; A=$2; B=$3
mkdir -p gpurun_out
for x in $A $B $A $B; do
  env $V=$x timeout -k 10 200 python bench.py --workload config5 --cpu-sample 0 > gpurun_out/ab_$x.json 2> gpurun_out/ab_$x.err || exit 1
  python -c "
import json; c=json.load(open('gpurun_out/ab_$x.json'))
print('$V=$x', c['correct'], {s:(v['gpu']['p50_us'], v['gpu']['p99_us'], v['concurrent_1_block_callers']['gpu']['p50_us'], v['concurrent_1_block_callers']['gpu']['p99_us'], v['concurrent_1_block_callers']['gpu']['blocks_per_s']) for s,v in c['shapes'].items()})"
done
