# pinned-input (streamed) verify: GPU tests of the host-buffer paths, then rates per batches/chunk size
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py -m gpu -x -q --timeout 120 --timeout-method thread -k "pipelined or config3 or sub_batch" > gpurun_out/t1.log 2>&1; rc=$?; tail -3 gpurun_out/t1.log; [ $rc -ne 0 ] && exit $rc
for nb in 1 2 3 4; do for c in 16 17; do MV_STREAM_BATCHES=$nb MV_STREAM_CHUNK_LOG2=$c timeout -k 10 120 python tools/pipe_probe.py 2>&1 | grep pinned | sed "s/^/batches=$nb /" || exit 1; done; done
