#!/bin/bash
# rocprofv3 evidence, round 2 final (run on the GPU box from the repo root):
#   kernel trace + stats: config 2 (2 streams = the bench default, and 1 stream), config 4
#   (1 stream), WAL; PMC passes (one counter group per run, no other tracing) on 1-stream runs.
# Usage: tools/profile_r02b.sh <tag>  -> gpurun_out/prof_<tag>/...
set -o pipefail
TAG=${1:-r02b}
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
C2="python bench.py --steps 5 --warmup 1 --cpu-sample 0 --no-e2e --sustain-repeats 0 --no-adversarial --no-config4 --no-wal"
C4="python bench.py --workload config4 --steps 3 --warmup 1 --cpu-sample 0 --streams 1"
WAL="python bench.py --workload wal --steps 3 --warmup 1 --cpu-sample 0"
run() {  # run <seconds> <log> <cmd...>
  local t=$1 log=$2; shift 2
  timeout -k 10 "$t" "$@" > "$log" 2>&1 || { echo "FAILED ($?): $*"; tail -5 "$log"; exit 1; }
}
run 300 "$OUT/trace.log" rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- $C2
run 300 "$OUT/trace1.log" rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace1" -o run -- $C2 --streams 1
run 300 "$OUT/trace_c4.log" rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_c4" -o run -- $C4
run 300 "$OUT/trace_wal.log" rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_wal" -o run -- $WAL
echo traces done
i=0
for group in \
  "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
  "SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_THREAD_CYCLES_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS" \
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LEVEL_WAVES" \
  "FETCH_SIZE" \
  "WRITE_SIZE"; do
  i=$((i+1))
  run 150 "$OUT/c2_pmc$i.log" timeout -s KILL 140 rocprofv3 --pmc $group --output-format csv -d "$OUT/c2/pmc$i" -o run -- $C2 --streams 1
  run 180 "$OUT/c4_pmc$i.log" timeout -s KILL 170 rocprofv3 --pmc $group --output-format csv -d "$OUT/c4/pmc$i" -o run -- $C4
  if [ $i -ge 4 ]; then
    run 180 "$OUT/wal_pmc$i.log" timeout -s KILL 170 rocprofv3 --pmc $group --output-format csv -d "$OUT/wal/pmc$i" -o run -- $WAL
  fi
  echo "pmc group $i done"
done
for k in k_bv_prep k_bv_bucket k_fine_sort k_part_scatter k_bv_final k_bv_reduce; do
  python tools/pmc_summary.py "$OUT/c2" $k --json "$OUT/pmc_c2_$k.json" > "$OUT/pmc_c2_$k.txt" || true
done
for k in k_b2_quad k_block_ingest k_bv_prep k_bv_bucket k_bv_keyacc k_bv_keypts; do
  python tools/pmc_summary.py "$OUT/c4" $k --json "$OUT/pmc_c4_$k.json" > "$OUT/pmc_c4_$k.txt" || true
done
for k in k_wal_crc k_wal_walk; do
  python tools/pmc_summary.py "$OUT/wal" $k --json "$OUT/pmc_wal_$k.json" > "$OUT/pmc_wal_$k.txt" || true
done
echo profile done
