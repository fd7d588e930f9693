# timeline of the config-5 latency path (64-block calls; kernel + memory-copy trace)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 python bench.py --workload config5 --cpu-sample 0 --batches 3000 --conc-seconds 0.5 > gpurun_out/c5_plain.json 2>gpurun_out/c5_plain.err || exit 1
timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/c5tl -o run -f csv -- python bench.py --workload config5 --cpu-sample 0 --batches 500 --conc-seconds 0.2 > gpurun_out/c5tl.log 2>&1 || exit 1
python tools/timeline.py gpurun_out/c5tl 300 > gpurun_out/c5_timeline.txt
python -c "
import json; d=json.load(open('gpurun_out/c5_plain.json'))
for s,v in d['shapes'].items(): print(s, v['gpu'])"
