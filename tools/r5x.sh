mkdir -p gpurun_out/r5s
C2="--cpu-sample 0 --no-e2e --sustain-repeats 0 --no-adversarial --no-config4 --no-wal --no-config5"
timeout -k 10 300 python -m pytest tests/test_gpu_batch.py -m gpu -x -q --timeout 240 --timeout-method thread -k bucket_forms > gpurun_out/r5s/t.log 2>&1 || { tail -30 gpurun_out/r5s/t.log; exit 1; }
tail -1 gpurun_out/r5s/t.log
for cfg in "20 3" "20 2" "20 4" "20 3" "20 2" "20 4" "600 3" "600 2" "600 4"; do set -- $cfg
  timeout -k 10 200 python bench.py --steps $1 --warmup 5 --streams $2 $C2 > gpurun_out/r5s/c2_$1_$2.json 2>/dev/null || exit 1
  python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print('c2',sys.argv[2],'streams',sys.argv[3],round(d['value']/1e6,2),d['ms_per_step'],d['correct'])" gpurun_out/r5s/c2_$1_$2.json $1 $2
done
