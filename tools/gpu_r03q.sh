#!/bin/bash
# Host-fed config 4: per-chunk host pack / enqueue times (MV_BLK_TRACE), pack threads 8 vs 16,
# chunk 256 vs 64 MiB.
set -o pipefail
mkdir -p gpurun_out
for cfg in "8 268435456" "16 268435456" "8 67108864"; do
  set -- $cfg
  MV_PACK_THREADS=$1 MV_BLK_CHUNK_BYTES=$2 MV_BLK_TRACE=1 timeout -k 10 300 python bench.py --workload config4 --batch 262144 --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/c4hf_$1_$2.json 2> gpurun_out/c4hf_$1_$2.err || { tail -5 gpurun_out/c4hf_$1_$2.err; exit 1; }
  python3 - <<PY
import json, re
d=json.load(open("gpurun_out/c4hf_$1_$2.json")); h=d["host_fed"]
rows=[l for l in open("gpurun_out/c4hf_$1_$2.err") if "[blk]" in l and "blocks" in l]
big=[l for l in rows if int(re.search(r'(\d+) blocks', l).group(1)) > 1000][-12:]
print("threads $1 chunk $2:", h["value"], h["frac_of_pcie_bound"], "h2d", h["h2d_GBps_pinned"])
for l in big[-4:]: print("   ", l.strip())
PY
done
