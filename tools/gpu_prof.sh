#!/bin/bash
# GPU-box profiling sequence: HBM ceiling, sharded virtual-rank tests, elim
# variant sweep, rocprofv3 kernel trace + stats of bench.py, then FETCH_SIZE and
# WRITE_SIZE in separate --pmc passes.  A fault / abort / timeout ends it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
fatal() { case "$1" in 0|1) return 1;; *) return 0;; esac; }
step() {  # step <limit_s> <log> <cmd...>
  local lim=$1 log=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$log" 2>&1
  local rc=$?
  echo "[$log] rc=$rc"; tail -${TAILN:-4} "gpurun_out/$log"
  if fatal $rc; then exit $rc; fi
  return 0
}
[ -n "${DO_CEIL:-1}" ] && [ "${DO_CEIL:-1}" != 0 ] && step 120 hbm_ceiling.log ./tools/hbm_ceiling
[ "${DO_TEST:-1}" != 0 ] && step 900 pytest_sel.log python -m pytest tests -m gpu -q ${PYTEST_K:-}
[ "${DO_TUNE:-1}" != 0 ] && TAILN=40 step 600 tune.log python tools/tune_elim.py
if [ "${DO_PROF:-1}" != 0 ]; then
  step 400 prof_bench.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench \
       --output-format csv -- python3 bench.py --steps 200 --cpu-seconds 0 ${BENCH_ARGS:-}
  step 400 pmc_fetch.log rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o f \
       --output-format csv -- python3 bench.py --steps 30 --warmup 5 --cpu-seconds 0 ${BENCH_ARGS:-}
  step 400 pmc_write.log rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o w \
       --output-format csv -- python3 bench.py --steps 30 --warmup 5 --cpu-seconds 0 ${BENCH_ARGS:-}
fi
exit 0
