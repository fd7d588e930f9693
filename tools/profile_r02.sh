#!/bin/bash
# rocprofv3 evidence, round 2 (run on the GPU box from the repo root):
#   kernel trace + stats: config 2 (2 streams = the bench default, and 1 stream), config 4 (1 stream)
#   PMC passes (one counter group per run, no other tracing) on 1-stream runs:
#     config 2 -> k_bv_prep, k_bv_bucket; config 4 -> k_b2_quad, k_block_ingest
# Usage: tools/profile_r02.sh <tag>  -> gpurun_out/prof_<tag>/...
set -eo pipefail
TAG=${1:-r02}
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
C2="python bench.py --steps 5 --warmup 1 --cpu-sample 0 --no-e2e --sustain-repeats 0 --no-adversarial --no-config4"
C4="python bench.py --workload config4 --steps 3 --warmup 1 --cpu-sample 0 --streams 1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- $C2 > "$OUT/trace.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace1" -o run -- $C2 --streams 1 > "$OUT/trace1.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_c4" -o run -- $C4 > "$OUT/trace_c4.log" 2>&1
i=0
for group in \
  "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
  "SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_THREAD_CYCLES_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS" \
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LEVEL_WAVES" \
  "FETCH_SIZE" \
  "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $group --output-format csv -d "$OUT/c2/pmc$i" -o run -- $C2 --streams 1 > "$OUT/c2_pmc$i.log" 2>&1
  timeout -s KILL 150 rocprofv3 --pmc $group --output-format csv -d "$OUT/c4/pmc$i" -o run -- $C4 > "$OUT/c4_pmc$i.log" 2>&1
done
cp -r "$OUT/trace1" "$OUT/c2/trace1"
cp -r "$OUT/trace_c4" "$OUT/c4/trace1"
for k in k_bv_prep k_bv_bucket k_fine_sort k_part_scatter k_bv_final k_bv_reduce; do
  python tools/pmc_summary.py "$OUT/c2" $k --json "$OUT/pmc_c2_$k.json" > "$OUT/pmc_c2_$k.txt" || true
done
for k in k_b2_quad k_block_ingest k_bv_prep k_bv_bucket k_bv_keyacc k_bv_keypts; do
  python tools/pmc_summary.py "$OUT/c4" $k --json "$OUT/pmc_c4_$k.json" > "$OUT/pmc_c4_$k.txt" || true
done
echo profile done
