#!/bin/bash
# Rehearses the driver's round-end GPU tier exactly: pytest -m gpu, then the smoke as a plain
# `python -c` whose stdout is a pipe (no -u, no debug environment). A Python-level watchdog
# (faulthandler) dumps every thread's stack if the smoke is still running after WD seconds, so
# a stall inside mv_destroy (a ctypes call) is told apart from one at interpreter exit (after
# finalisation faulthandler is gone and the log just ends).
#   tools/smoke_driver.sh TAG [REPS]  -> gpurun_out/TAG/
set -o pipefail
TAG=${1:?tag}
REPS=${2:-3}
WD=${WD:-60}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 600 python -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { echo "pytest FAILED"; tail -20 "$OUT/pytest.log"; exit 1; }
  tail -1 "$OUT/pytest.log"
fi
for r in $(seq 1 "$REPS"); do
  t0=$(date +%s.%N)
  timeout -k 10 120 python -c "
import faulthandler, sys
faulthandler.dump_traceback_later($WD, exit=True)
import __graft_entry__ as g
g.smoke()
print('__SMOKE_OK__')
" 2>&1 | cat > "$OUT/smoke_$r.log"
  rc=$?
  t1=$(date +%s.%N)
  echo "smoke $r rc=$rc $(python3 -c "print(round($t1-$t0,2))") s: $(tail -1 "$OUT/smoke_$r.log")"
  [ $rc -ne 0 ] && { tail -40 "$OUT/smoke_$r.log"; exit 1; }
done
exit 0
