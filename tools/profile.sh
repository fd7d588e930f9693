#!/bin/bash
# rocprofv3 evidence for the verify pipeline (run on the GPU box from the repo root):
#   1. kernel trace + stats (average duration per kernel) of the default bench command
#   2. PMC passes, one counter group per run (no sys/runtime trace with --pmc), on the
#      single-stream batch bench so per-dispatch counters are not mixed by overlap
# Usage: tools/profile.sh <tag>   -> gpurun_out/prof_<tag>/...
set -eo pipefail
TAG=${1:-r01}
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
TRACE_BENCH="python bench.py --steps 5 --warmup 1 --cpu-sample 0 --no-e2e"
PMC_BENCH="python bench.py --steps 3 --warmup 1 --cpu-sample 0 --no-e2e --streams 1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- $TRACE_BENCH > "$OUT/trace.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace1" -o run -- $PMC_BENCH > "$OUT/trace1.log" 2>&1
i=0
for group in \
  "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
  "SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_THREAD_CYCLES_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS" \
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LEVEL_WAVES" \
  "FETCH_SIZE" \
  "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $group --output-format csv -d "$OUT/pmc$i" -o run -- $PMC_BENCH > "$OUT/pmc$i.log" 2>&1
done
cp -r "$OUT/trace1" "$OUT/trace_single_stream"
for k in k_bv_prep k_bv_bucket k_fine_sort k_part_scatter k_bv_final; do
  python tools/pmc_summary.py "$OUT" $k --json "$OUT/pmc_$k.json" > "$OUT/pmc_$k.txt"
done
echo profile done
