#!/bin/bash
# Windowed elimination on the box: window parity tests, then bench at several
# window sizes and a rocprofv3 kernel summary at WIN_PROF.  Each GPU step has
# its own limit; a fault / abort / timeout ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/win
fatal() { case "$1" in 0|1) return 1;; *) return 0;; esac; }
step() { local lim=$1 log=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/win/$log" 2>&1
  local rc=$?; echo "[$log] rc=$rc"; tail -${TAILN:-3} "gpurun_out/win/$log" | cut -c1-600
  if fatal $rc; then exit $rc; fi; }
TAILN=15 step ${PYTEST_LIMIT:-600} pytest_window.log python -m pytest tests -m gpu -q -x ${PYTEST_FILES:-tests/test_gpu_window.py}
for K in ${WINS:-0 4 8 16}; do
  step 300 bench_k$K.log python bench.py --window $K --steps ${STEPS:-256} --cpu-seconds 0
done
if [ -n "${WIN_PROF:-}" ]; then
  step 400 rocprof_k.log rocprofv3 --kernel-trace --stats -d gpurun_out/win/prof -o w --output-format csv -- python3 bench.py --window $WIN_PROF --steps ${STEPS:-256} --cpu-seconds 0
fi
exit 0
