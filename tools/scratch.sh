set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ks1 -o run -- python bench.py --steps 5 --warmup 1 --cpu-sample 0 --no-e2e --sustain-repeats 0 --no-adversarial --no-config4 --no-wal --streams 1 > gpurun_out/ks1.log 2>&1 || exit 1
python -c "
import csv
for r in csv.DictReader(open('gpurun_out/ks1/run_kernel_stats.csv')):
    print(r['Name'][:50], r['Calls'], round(float(r['AverageNs'])/1e3,1))"
