mkdir -p gpurun_out/r5bc
C2="--cpu-sample 0 --no-e2e --sustain-repeats 0 --no-adversarial --no-config4 --no-wal --no-config5"
for cfg in "20 1 3" "20 2 3" "20 1 3" "20 2 3" "600 1 3" "600 2 3" "600 2 4" "600 1 3" "600 2 3"; do set -- $cfg
  MV_PREP_CHAIN=$2 timeout -k 10 200 python bench.py --steps $1 --warmup 5 --streams $3 $C2 > gpurun_out/r5bc/c2_$1_$2_$3.json 2>/dev/null || exit 1
  python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print('c2',sys.argv[2],'chain',sys.argv[3],'streams',sys.argv[4],round(d['value']/1e6,2),d['ms_per_step'],d['correct'])" gpurun_out/r5bc/c2_$1_$2_$3.json $1 $2 $3
done
