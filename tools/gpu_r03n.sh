#!/bin/bash
# Host-side cost of one online pass (MV_BLK_TRACE): pack / copy / kernel-enqueue microseconds.
set -o pipefail
mkdir -p gpurun_out
MV_BLK_TRACE=1 timeout -k 10 200 python bench.py --workload config5 --cpu-sample 0 --batches 300 --conc-seconds 0.5 > gpurun_out/c5_trace.json 2> gpurun_out/c5_trace.err || { tail -5 gpurun_out/c5_trace.err; exit 1; }
grep "\[blk\]" gpurun_out/c5_trace.err | tail -400 | python3 -c "
import sys, re, statistics as S
rows=[l for l in sys.stdin]
for key in ('pack','h2d','kernels'):
    v=[float(re.search(key+r' ([0-9.]+)', l).group(1)) for l in rows if re.search(key+r' ([0-9.]+)', l)]
    print(key, 'median', S.median(v), 'p90', sorted(v)[int(0.9*len(v))], 'n', len(v))
blocks=[int(re.search(r'(\d+) blocks', l).group(1)) for l in rows]
print('blocks per pass median', S.median(blocks))
"
