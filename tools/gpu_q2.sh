#!/bin/bash
# hash-kernel A/B: GPU tests of the hash paths, config-4 bench, one LDS PMC pass on config 4
set -o pipefail
TAG=${1:-q2}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_primitives.py tests/test_gpu_blocks.py tests/test_gpu_ingest.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/$TAG/pytest.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED|Error" gpurun_out/$TAG/pytest.log | head -30; exit $rc; }
timeout -k 10 300 python bench.py --workload config4 --cpu-sample 0 > gpurun_out/$TAG/c4.json 2> gpurun_out/$TAG/c4.err || exit 1
timeout -k 10 300 python bench.py --workload config4 --cpu-sample 0 --streams 1 > gpurun_out/$TAG/c4_s1.json 2> gpurun_out/$TAG/c4_s1.err || exit 1
C4="python bench.py --workload config4 --steps 3 --warmup 1 --cpu-sample 0 --streams 1"
timeout -s KILL 150 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_WAVES --output-format csv -d gpurun_out/$TAG/pmc -o run -- $C4 > gpurun_out/$TAG/pmc.log 2>&1 || exit 1
python tools/pmc_summary.py gpurun_out/$TAG/pmc k_b2_quad > gpurun_out/$TAG/pmc_b2.txt || true
python - <<PY
import json
for f in ("c4","c4_s1"):
    d=json.load(open("gpurun_out/$TAG/%s.json"%f)); d=d.get("config4") or d
    print(f, round(d["value"]/1e6,1), "M/s", d["correct"], d["pipeline"]["stage_ms"])
PY
cat gpurun_out/$TAG/pmc_b2.txt
