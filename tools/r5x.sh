mkdir -p gpurun_out/r5z
C2="--cpu-sample 0 --no-e2e --sustain-repeats 0 --no-adversarial --no-config4 --no-wal --no-config5"
timeout -k 10 400 python -m pytest tests/test_gpu_batch.py tests/test_gpu_verify.py tests/test_gpu_blocks.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r5z/t.log 2>&1 || { tail -30 gpurun_out/r5z/t.log; exit 1; }
tail -1 gpurun_out/r5z/t.log
for cfg in "20 1" "20 0" "20 32" "20 128" "20 1" "20 0" "600 1" "600 0"; do set -- $cfg
  MV_BUCKET_BAL=$2 timeout -k 10 200 python bench.py --steps $1 --warmup 5 $C2 > gpurun_out/r5z/c2_$1_$2.json 2>/dev/null || exit 1
  python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print('c2',sys.argv[2],'bal',sys.argv[3],round(d['value']/1e6,2),d['ms_per_step'],d['correct'],d['parity_sha256'],d['roofline']['stage_ms_one_stream'])" gpurun_out/r5z/c2_$1_$2.json $1 $2
done
