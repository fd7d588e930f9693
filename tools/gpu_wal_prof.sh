#!/bin/bash
# WAL row (f4): full-size bench line, kernel trace, PMC passes for k_wal_crc / k_wal_walk
set -o pipefail
TAG=${1:-walp}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --workload wal --steps 10 --warmup 2 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
W="python bench.py --workload wal --steps 3 --warmup 1 --cpu-sample 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace1 -o run -- $W > $OUT/trace.log 2>&1 || exit 1
i=0
for group in "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS" \
  "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $group --output-format csv -d $OUT/pmc$i -o run -- $W > $OUT/pmc$i.log 2>&1 || { echo "pmc $i failed"; exit 1; }
done
for k in k_wal_crc k_wal_walk; do python tools/pmc_summary.py $OUT $k --json $OUT/pmc_wal_$k.json > $OUT/pmc_wal_$k.txt || true; done
cat $OUT/pmc_wal_k_wal_crc.txt
