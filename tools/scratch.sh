set -o pipefail
MV_BLK_TRACE=1 timeout -k 10 120 python bench.py --workload config5 --cpu-sample 0 --batches 300 --conc-seconds 0.1 > gpurun_out/c5t.json 2> gpurun_out/c5t.err || exit 1
grep "\[blk\] 64 blocks" gpurun_out/c5t.err | tail -400 | awk 'NR%50==0'
