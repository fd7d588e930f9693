#!/bin/bash
# Final round bench lines: default config-2 line, config-4 block throughput, config-5 latency.
set -o pipefail
TAG=${1:-r01f2}
mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/bench_c2_$TAG.json 2> gpurun_out/bench_c2_$TAG.err || exit 1
cat gpurun_out/bench_c2_$TAG.json
timeout -k 10 300 python bench.py --workload config4 > gpurun_out/bench_c4_$TAG.json 2> gpurun_out/bench_c4_$TAG.err || exit 1
cat gpurun_out/bench_c4_$TAG.json
timeout -k 10 400 python bench.py --workload config5 > gpurun_out/bench_c5_$TAG.json 2> gpurun_out/bench_c5_$TAG.err || exit 1
cat gpurun_out/bench_c5_$TAG.json
