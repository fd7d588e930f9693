set -o pipefail
MV_LIB=$PWD/mysticeti_amd/_build/glds/libmysti_verify.so timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_blocks.py -m gpu -x -q --timeout 200 --timeout-method thread 2>&1 | tail -1
bash tools/ab.sh main glds main glds || exit 1
for v in main glds; do
  if [ $v = main ]; then unset MV_LIB; else export MV_LIB=$PWD/mysticeti_amd/_build/glds/libmysti_verify.so; fi
  timeout -k 10 300 python bench.py --workload config4 --cpu-sample 0 > gpurun_out/c4_$v.json 2>/dev/null || exit 1
  python -c "
import json; d=json.load(open('gpurun_out/c4_$v.json')); d=d.get('config4') or d
print('c4 $v', round(d['value']/1e6,1), d['correct'], d['pipeline']['stage_ms']['bucket'])"
done
