#!/bin/bash
# GPU-box sequence: smoke -> parity tests -> short bench.  Each GPU step has
# its own time limit; a fault / abort / timeout ends the script there.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
fatal() { case "$1" in 0|1) return 1;; *) return 0;; esac; }

timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
if fatal $rc; then exit $rc; fi

timeout -k 10 ${PYTEST_LIMIT:-900} python -m pytest tests -m gpu -q ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -25 gpurun_out/pytest_gpu.log
if fatal $rc; then exit $rc; fi

if [ "${SKIP_BENCH:-0}" = "0" ]; then
  timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
  rc=$?; echo "bench rc=$rc"; tail -5 gpurun_out/bench.log
fi
exit $rc
