#!/bin/bash
# full GPU suite, default bench line, config-5 latency (queue + pooled CPU)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_r02d.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_r02d.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED|Error" gpurun_out/pytest_r02d.log | head -30; exit $rc; }
timeout -k 10 300 python bench.py > gpurun_out/bench_r02d.json 2> gpurun_out/bench_r02d.err || { tail gpurun_out/bench_r02d.err; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/bench_r02d.json"))
print("value", round(d["value"]/1e6,1), "correct", d["correct"], "frac", d["roofline"]["frac"], "frac_8d", d["roofline"]["frac_8d"]["value"])
print("sustained", d["sustained"]["median"]/1e6, "adv", {k: (round(v["value"]/1e6,1), v["ratio_to_all_valid"]) for k, v in d["adversarial"].items() if k != "note"})
print("cpu", d["cpu_baseline"]["value"], d["cpu_baseline"]["cores"], d["cpu_baseline"]["cores_source"], "e2e", d["end_to_end"]["value"]/1e6)
PY
timeout -k 10 300 python bench.py --workload config5 --batches 3000 --conc-seconds 2 > gpurun_out/c5_r02d.json 2> gpurun_out/c5_r02d.err || { tail gpurun_out/c5_r02d.err; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/c5_r02d.json"))
for sh, r in d["shapes"].items():
    print(sh, {k: (v["p50_us"], v["p99_us"]) for k, v in r.items() if isinstance(v, dict) and "p50_us" in v})
    print("  conc", json.dumps(r["concurrent_1_block_callers"]))
PY
