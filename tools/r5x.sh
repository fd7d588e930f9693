mkdir -p gpurun_out/r5m
timeout -k 10 300 python -m pytest tests/test_gpu_batch.py -m gpu -x -q --timeout 240 --timeout-method thread -k "streaming_msm or bucket_forms or streamed or pipelined or valid_batches" > gpurun_out/r5m/t2.log 2>&1 || { tail -30 gpurun_out/r5m/t2.log; exit 1; }
tail -1 gpurun_out/r5m/t2.log
