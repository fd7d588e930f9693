#!/bin/bash
# One parameterised GPU driver for every measurement this repo takes on the box (replaces the
# round-2/3 one-shot gpu_r0x*.sh scripts).
#
#   tools/gpu.sh TAG TASK [TASK ...]        -> gpurun_out/TAG/
#
# Tasks run in order; the first failure (or time limit) ends the script, nothing more touches
# the GPU after it. Every GPU step runs under its own `timeout -k 10`.
#
#   tests[:K]        pytest -m gpu (K: a -k expression)
#   smoke            __graft_entry__.smoke()
#   bench            the driver's default line: bench.py --gpus 1 --steps 20 --warmup 5
#   bench100         the default line at 100 steps (steady-state cross-check of `bench`)
#   c2[:ARGS]        config-2 line only (no legs); ARGS (comma-separated) appended
#   c4[:ARGS]        --workload config4 (2^21 blocks, 20 steps); ARGS appended
#   c5               --workload config5
#   wal              --workload wal
#   gpus2            --gpus 2 rehearsal (both ranks on the one GPU)
#   ab:V[:ARGS]      config-2 line, product library vs experiment build V (MV_LIB), 2 interleaved reps
#   abc4:V[:ARGS]    the same on config 4
#   env:K=V          export K=V for the tasks that follow (SUF=x: later bench outputs are named <task>x.json)
#   e2e[:ENV=V,..]   tools/e2e_probe.py (pinned end-to-end signatures) under these settings
#   benchtrace       the driver's bench command under rocprofv3 --kernel-trace --stats
#   h2d              tools/h2d_probe.py: pinned H2D rates (whole arrays, chunks, two streams)
#   e2etrace         tools/e2e_probe.py with two callers (MV_PROBE_TWO) under kernel + memory-copy trace
#   trace:W          rocprofv3 --kernel-trace --stats of workload W in {c2, c2s1, c2single, c4, c4s1, c5, wal}
#   pmc:W[:KERNELS]  separate --pmc passes (one counter group per run) of W in {c2s1, c4s1, wal} and
#                    tools/pmc_summary.py for each kernel (comma-separated)
#   pmcg:W:K:C1,C2.. ONE --pmc pass of W with the counters C1,C2,.. (one block's limits), per kernel K
#   avail            rocprofv3 --list-avail (the TCC_/TCP_ counter names in the output)
#   teardown         tools/teardown_probe.py plain, then under rocprofv3 hip + kernel + memory-copy
#                    trace (/proc maps at exit); run it LAST in a call (it may end in a teardown fault)
set -o pipefail
TAG=${1:?tag}
shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1

C2ONLY="--cpu-sample 0 --no-e2e --sustain-repeats 0 --no-adversarial --no-config4 --no-wal --no-config5"
declare -A W=(
  [c2]="python bench.py --steps 5 --warmup 1 $C2ONLY"
  [c2s1]="python bench.py --steps 5 --warmup 1 --streams 1 $C2ONLY"
  [c2single]="python bench.py --steps 5 --warmup 1 --streams 1 --path single $C2ONLY"
  [c4]="python bench.py --workload config4 --steps 6 --warmup 4 --cpu-sample 0 --host-fed-blocks 0 --batch 1048576"
  [c4s1]="python bench.py --workload config4 --steps 3 --warmup 1 --cpu-sample 0 --streams 1 --host-fed-blocks 0 --batch 1048576"
  [c5]="python bench.py --workload config5 --cpu-sample 0 --batches 1000 --conc-seconds 0.3"
  [wal]="python bench.py --workload wal --steps 3 --warmup 1 --cpu-sample 0"
)
PMC_GROUPS=(
  "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
  "SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_THREAD_CYCLES_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS"
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LEVEL_WAVES"
  "FETCH_SIZE"
  "WRITE_SIZE"
)

run() {  # run <seconds> <log> <cmd...>: stop the script on failure
  local t=$1 log=$2
  shift 2
  timeout -k 10 "$t" "$@" > "$log" 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then
    echo "FAILED rc=$rc: $*"
    tail -8 "$log"
    exit 1
  fi
}
line() {  # line <json>: one-line digest of a bench JSON
  python3 tools/line_digest.py "$1"
}

for T in "$@"; do
  name=${T%%:*}
  arg=""
  [ "$T" != "$name" ] && arg=${T#*:}
  case $name in
    tests)
      K=()
      [ -n "$arg" ] && K=(-k "$arg")
      run 900 "$OUT/pytest_gpu.log" python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread "${K[@]}"
      tail -1 "$OUT/pytest_gpu.log" ;;
    smoke)
      # exactly the driver's command: no -u, no debug environment (a stall then shows as it
      # would to the driver; tools/smoke_driver.sh adds a stack-dumping watchdog)
      run 150 "$OUT/smoke.log" python -c "import __graft_entry__ as g; g.smoke(); print('__SMOKE_OK__')"
      tail -1 "$OUT/smoke.log" ;;
    bench)
      timeout -k 10 900 python bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench$SUF.json" 2> "$OUT/bench$SUF.err" || { echo "bench FAILED"; tail -8 "$OUT/bench$SUF.err"; exit 1; }
      line "$OUT/bench$SUF.json" ;;
    bench100)
      timeout -k 10 900 python bench.py --steps 100 --warmup 5 > "$OUT/bench100$SUF.json" 2> "$OUT/bench100$SUF.err" || { echo "bench100 FAILED"; tail -8 "$OUT/bench100$SUF.err"; exit 1; }
      line "$OUT/bench100$SUF.json" ;;
    c2)
      timeout -k 10 300 python bench.py --steps 600 --warmup 10 $C2ONLY ${arg//,/ } > "$OUT/c2$SUF.json" 2> "$OUT/c2$SUF.err" || { echo "c2 FAILED"; tail -8 "$OUT/c2$SUF.err"; exit 1; }
      line "$OUT/c2$SUF.json" ;;
    c4)
      timeout -k 10 600 python bench.py --workload config4 --steps 20 --warmup 5 --cpu-sample 0 ${arg//,/ } > "$OUT/c4$SUF.json" 2> "$OUT/c4$SUF.err" || { echo "c4 FAILED"; tail -8 "$OUT/c4$SUF.err"; exit 1; }
      line "$OUT/c4$SUF.json" ;;
    c5)
      timeout -k 10 600 python bench.py --workload config5 --cpu-sample 0 --batches 2000 --conc-seconds 2 ${arg//,/ } > "$OUT/c5$SUF.json" 2> "$OUT/c5$SUF.err" || { echo "c5 FAILED"; tail -8 "$OUT/c5$SUF.err"; exit 1; }
      line "$OUT/c5$SUF.json" ;;
    wal)
      timeout -k 10 600 python bench.py --workload wal --steps 20 --warmup 2 --cpu-sample 0 > "$OUT/wal$SUF.json" 2> "$OUT/wal$SUF.err" || { echo "wal FAILED"; tail -8 "$OUT/wal$SUF.err"; exit 1; }
      line "$OUT/wal$SUF.json" ;;
    gpus2)
      timeout -k 10 600 python bench.py --gpus 2 --steps 20 --warmup 5 --no-config5 --host-fed-blocks 0 --cpu-sample 0 --no-e2e --sustain-repeats 1 > "$OUT/gpus2$SUF.json" 2> "$OUT/gpus2$SUF.err" || { echo "gpus2 FAILED"; tail -8 "$OUT/gpus2$SUF.err"; exit 1; }
      line "$OUT/gpus2$SUF.json" ;;
    ab|abc4)
      V=${arg%%:*}
      A=""
      [ "$arg" != "$V" ] && A=${arg#*:}
      L=$GRAFT_REPO_ROOT/mysticeti_amd/_build/$V/libmysti_verify.so
      [ -f "$L" ] || { echo "no variant build $L"; exit 1; }
      for rep in 1 2; do
        for lib in product "$V"; do
          if [ $lib = product ]; then ML=""; else ML=$L; fi
          if [ $name = ab ]; then
            CMD="python bench.py --steps 600 --warmup 10 $C2ONLY ${A//,/ }"
          else
            CMD="python bench.py --workload config4 --steps 20 --warmup 5 --cpu-sample 0 --host-fed-blocks 0 ${A//,/ }"
          fi
          # exit 1 = verdicts wrong (an experiment build may compute garbage on purpose): kept
          MV_LIB=$ML timeout -k 10 400 $CMD > "$OUT/${name}_${lib}_$rep.json" 2> "$OUT/${name}_${lib}_$rep.err"
          rc=$?
          if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "$name $lib FAILED rc=$rc"; tail -8 "$OUT/${name}_${lib}_$rep.err"; exit 1; fi
          echo -n "rep $rep $lib: "
          line "$OUT/${name}_${lib}_$rep.json"
        done
      done ;;
    env)  # env:K=V -- exported for the tasks after it
      export "$arg"
      echo "env $arg" ;;
    e2e)  # e2e[:ENV=V,ENV=V]: the pinned end-to-end probe under these environment settings
      (export ${arg//,/ }; timeout -k 10 300 python tools/e2e_probe.py) >> "$OUT/e2e.log" 2>&1 || { echo "e2e FAILED"; tail -5 "$OUT/e2e.log"; exit 1; }
      tail -1 "$OUT/e2e.log" ;;
    benchtrace)  # the driver's bench command under rocprofv3 --kernel-trace --stats (the roofline's source)
      run 900 "$OUT/benchtrace.log" rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/benchtrace" -o run -- python bench.py --gpus 1 --steps 20 --warmup 5
      grep -E '^\{' "$OUT/benchtrace.log" | tail -1 | cut -c1-200
      python3 tools/trace_top.py "$OUT/benchtrace" ;;
    h2d)  # tools/h2d_probe.py: pinned H2D rates in the streamed path's copy shapes
      run 300 "$OUT/h2d.log" python tools/h2d_probe.py
      grep "^h2d" "$OUT/h2d.log" ;;
    e2etrace)  # the pinned probe with two callers, under a kernel + memory-copy trace (timeline)
      (export MV_PROBE_TWO=1; run 300 "$OUT/e2etrace.log" rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$OUT/e2etrace" -o run -- python tools/e2e_probe.py) || exit 1
      grep -E "two callers|e2e pinned" "$OUT/e2etrace.log" ;;
    trace)
      cmd=${W[$arg]}
      [ -n "$cmd" ] || { echo "unknown workload $arg"; exit 1; }
      run 400 "$OUT/trace_$arg.log" rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_$arg" -o run -- $cmd
      python3 tools/trace_top.py "$OUT/trace_$arg" ;;
    pmc)
      wl=${arg%%:*}
      ks=""
      [ "$arg" != "$wl" ] && ks=${arg#*:}
      cmd=${W[$wl]}
      [ -n "$cmd" ] || { echo "unknown workload $wl"; exit 1; }
      mkdir -p "$OUT/pmc_$wl"
      # config 4: one parse and one hash launch per call (no two halves), so every launch of a
      # kernel covers the same 2^20 blocks and the per-launch averages are per 2^20 blocks
      [ "$wl" = c4s1 ] && export MV_BLK_PIPE=0
      run 400 "$OUT/pmc_$wl/trace.log" rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/pmc_$wl/trace1" -o run -- $cmd
      i=0
      for group in "${PMC_GROUPS[@]}"; do
        i=$((i + 1))
        run 200 "$OUT/pmc_$wl/pmc$i.log" timeout -s KILL 190 rocprofv3 --pmc $group --output-format csv -d "$OUT/pmc_$wl/pmc$i" -o run -- $cmd
      done
      for k in ${ks//,/ }; do
        python3 tools/pmc_summary.py "$OUT/pmc_$wl" "$k" --json "$OUT/pmc_${wl}_$k.json" > "$OUT/pmc_${wl}_$k.txt" || true
        grep -E "valu_issue|WAIT_INST|clock|fetch_GB|write_GB|kernel_avg|LDS_BANK" "$OUT/pmc_${wl}_$k.txt" | sed "s/^/$k /"
      done ;;
    pmcg)  # pmcg:W:KERNELS:C1,C2,..: ONE extra --pmc pass with these counters (within one block's
           # limits: at most 4 TCC_, 8 SQ_ ...), summarised per kernel
      wl=${arg%%:*}
      rest=${arg#*:}
      ks=${rest%%:*}
      ctrs=${rest#*:}
      cmd=${W[$wl]}
      [ -n "$cmd" ] || { echo "unknown workload $wl"; exit 1; }
      [ "$wl" = c4s1 ] && export MV_BLK_PIPE=0
      g=$OUT/pmcg_$wl${SUF:-}
      mkdir -p "$g"
      [ -d "$g/trace1" ] || run 400 "$g/trace.log" rocprofv3 --kernel-trace --stats --output-format csv -d "$g/trace1" -o run -- $cmd
      n=$(ls -d "$g"/pmc* 2>/dev/null | wc -l)
      run 200 "$g/pmc$n.log" timeout -s KILL 190 rocprofv3 --pmc ${ctrs//,/ } --output-format csv -d "$g/pmc$n" -o run -- $cmd
      for k in ${ks//,/ }; do
        python3 tools/pmc_summary.py "$g" "$k" > "$OUT/pmcg_${wl}${SUF:-}_$k.txt" || true
        sed "s/^/$k /" "$OUT/pmcg_${wl}${SUF:-}_$k.txt"
      done ;;
    avail)
      run 120 "$OUT/avail.txt" rocprofv3 --list-avail
      grep -oE "(TCC|TCP)_[A-Z0-9_]+" "$OUT/avail.txt" | sort -u | tr '\n' ' ' > "$OUT/avail_tcc.txt" || true
      cut -c1-4000 "$OUT/avail_tcc.txt" ;;
    teardown)
      run 300 "$OUT/teardown_plain.log" python tools/teardown_probe.py "$OUT/maps_plain.txt"
      echo "plain: ok"
      timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace -d "$OUT/teardown_prof" -o run -f csv -- python tools/teardown_probe.py "$OUT/maps_prof.txt" > "$OUT/teardown_prof.log" 2>&1
      echo "under rocprofv3: rc=$?"
      tail -25 "$OUT/teardown_prof.log" ;;
    *)
      echo "unknown task $T"
      exit 1 ;;
  esac
done
echo "gpu.sh $TAG done"
