#!/bin/bash
# GPU iteration loop: parity tests, then the bench for both verify occupancy variants.
set -o pipefail
timeout -k 10 300 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED" gpurun_out/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 200 python bench.py --cpu-sample 0 --no-e2e > gpurun_out/b_occ2.json || exit 1
MV_VERIFY_OCC=1 timeout -k 10 200 python bench.py --cpu-sample 0 --no-e2e > gpurun_out/b_occ1.json || exit 1
python - <<'PY'
import json
for f in ["gpurun_out/b_occ2.json", "gpurun_out/b_occ1.json"]:
    d = json.load(open(f))
    print(f, d["value"], d["roofline"]["kernel_ms"], d["correct"], d["parity_sha256"])
PY
