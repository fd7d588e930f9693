set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_blocks.py tests/test_gpu_comb.py tests/test_gpu_engine.py -m gpu -x -q --timeout 200 --timeout-method thread 2>&1 | tail -3 || exit 1
timeout -k 10 120 python bench.py --workload config5 --cpu-sample 0 --batches 3000 --conc-seconds 0.5 > gpurun_out/c5_split.json 2>gpurun_out/c5_split.err || exit 1
MV_COMB_SPLIT_BYTES=0 timeout -k 10 120 python bench.py --workload config5 --cpu-sample 0 --batches 3000 --conc-seconds 0.5 > gpurun_out/c5_fused.json 2>>gpurun_out/c5_split.err || exit 1
python -c "
import json
for f in ('split','fused'):
    d=json.load(open(f'gpurun_out/c5_{f}.json'))
    for s,v in d['shapes'].items(): print(f, s, v['gpu'], d['correct'])"
