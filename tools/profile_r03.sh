#!/bin/bash
# Round-3 final evidence, part B: rocprofv3 kernel traces (config 2 on 2 streams and 1, config 4
# on 1 stream, config 5) and PMC passes (one counter group per run, nothing else traced).
#   tools/profile_r03.sh -> gpurun_out/prof_r03/
set -o pipefail
OUT=gpurun_out/prof_r03
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
C2="python bench.py --steps 5 --warmup 1 --cpu-sample 0 --no-e2e --sustain-repeats 0 --no-adversarial --no-config4 --no-wal --no-config5"
C4="python bench.py --workload config4 --steps 3 --warmup 1 --cpu-sample 0 --streams 1 --host-fed-blocks 0"
C5="python bench.py --workload config5 --cpu-sample 0 --batches 1000 --conc-seconds 0.3"
run() {  # run <seconds> <log> <cmd...>
  local t=$1 log=$2; shift 2
  timeout -k 10 "$t" "$@" > "$log" 2>&1 || { echo "FAILED ($?): $*"; tail -5 "$log"; exit 1; }
}
run 300 "$OUT/trace.log" rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- $C2
run 300 "$OUT/trace1.log" rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace1" -o run -- $C2 --streams 1
run 300 "$OUT/trace_c4.log" rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_c4" -o run -- $C4
run 300 "$OUT/trace_c5.log" rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_c5" -o run -- $C5
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
  echo "pmc group $i done"
done
cp -r "$OUT/trace1" "$OUT/c2/trace1"
cp -r "$OUT/trace_c4" "$OUT/c4/trace1"
for k in k_bv_prep k_bv_bucket k_fine_sort k_part_scatter k_bv_final k_bv_reduce; do
  python tools/pmc_summary.py "$OUT/c2" $k --json "$OUT/pmc_c2_$k.json" > "$OUT/pmc_c2_$k.txt" || true
done
for k in k_b2_lane k_block_ingest k_bv_prep k_bv_bucket; do
  python tools/pmc_summary.py "$OUT/c4" $k --json "$OUT/pmc_c4_$k.json" > "$OUT/pmc_c4_$k.txt" || true
done
echo profile done
