#!/bin/bash
# Session-3 probes: pinned host-buffer verify chunk sizes; WAL crc rows in flight (4 / 8 / 16).
set -o pipefail
mkdir -p gpurun_out
for C in 17 18 19; do
  MV_PIPE_CHUNK_LOG2=$C timeout -k 10 180 python tools/pipe_probe.py > gpurun_out/s3b_pipe_$C.log 2>&1 || { tail -20 gpurun_out/s3b_pipe_$C.log; exit 1; }
  cat gpurun_out/s3b_pipe_$C.log
done
for V in walrows4 walrows16 main; do
  if [ $V = main ]; then L=""; else L=mysticeti_amd/_build/$V/libmysti_verify.so; fi
  MV_LIB=$L timeout -k 10 200 python bench.py --workload wal --steps 10 --warmup 2 --cpu-sample 0 > gpurun_out/s3b_wal_$V.json 2> gpurun_out/s3b_wal_$V.err || { tail -20 gpurun_out/s3b_wal_$V.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/s3b_wal_$V.json'));print('$V', d['value'], d['stage_ms'], d['correct'])"
done
# config-5 timeline: kernel + copy trace of the latency bench (GPU legs only)
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/s3b_c5trace -o run -- python bench.py --workload config5 --cpu-sample 0 --batches 2000 --conc-seconds 1 > gpurun_out/s3b_c5trace.log 2>&1 || { tail -20 gpurun_out/s3b_c5trace.log; exit 1; }
echo c5 trace done
