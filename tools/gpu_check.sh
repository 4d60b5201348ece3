#!/bin/bash
# GPU-box sequence: smoke -> parity tests -> short bench.  Each GPU step has
# its own time limit; a fault / abort / timeout ends the script there.
# Output under gpurun_out/$OUT (default chk).  PYTEST_ARGS selects tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-chk}
mkdir -p $O
fatal() { case "$1" in 0|1) return 1;; *) return 0;; esac; }

timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 $O/smoke.log
if fatal $rc; then exit $rc; fi

timeout -k 10 ${PYTEST_LIMIT:-900} python -u -m pytest tests -m gpu -x -q --timeout 120 \
  --timeout-method thread ${PYTEST_ARGS:-} > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -25 $O/pytest_gpu.log
if fatal $rc; then exit $rc; fi
[ $rc != 0 ] && exit $rc

if [ "${SKIP_BENCH:-0}" = "0" ]; then
  timeout -k 10 300 python bench.py ${BENCH_ARGS:-} > $O/bench.log 2>&1
  rc=$?; echo "bench rc=$rc"; tail -5 $O/bench.log
fi
exit $rc
