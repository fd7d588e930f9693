#!/bin/bash
# PMC passes (one counter group per run) over the config-4 bench, summarised for one kernel.
#   tools/pmc_ingest.sh <tag> [kernel]
set -o pipefail
TAG=${1:-ing}; K=${2:-k_block_ingest}
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
CMD="python bench.py --workload config4 --batch 262144 --steps 2 --warmup 1 --cpu-sample 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace1 -o run -- $CMD > $OUT/trace.log 2>&1 || exit 1
i=0
for group in \
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD" \
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_WR" \
  "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $group --output-format csv -d $OUT/pmc$i -o run -- $CMD > $OUT/pmc$i.log 2>&1 || { tail -5 $OUT/pmc$i.log; exit 1; }
done
python tools/pmc_summary.py $OUT $K --json $OUT/pmc_$K.json
