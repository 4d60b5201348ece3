#!/bin/bash
# tests -> bench -> sweep, each step time-limited; stop at the first fault.
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
fatal() { case "$1" in 0|1) return 1;; *) return 0;; esac; }
timeout -k 10 900 python -m pytest tests -m gpu -q ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_all.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_all.log; if fatal $rc; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 400 --cpu-seconds ${CPU_S:-0} > gpurun_out/bench_default.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_default.log | cut -c1-200; if fatal $rc; then exit $rc; fi
if [ "${DO_TUNE:-1}" != 0 ]; then
  timeout -k 10 600 python tools/tune_elim.py > gpurun_out/tune.log 2>&1
  rc=$?; echo "tune rc=$rc"; if fatal $rc; then exit $rc; fi
fi
exit 0
