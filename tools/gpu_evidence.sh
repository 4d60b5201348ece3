#!/bin/bash
# Round evidence: full parity suite, config 2/5 timings, bench (with CPU
# baseline), rocprofv3 kernel trace + stats of the same bench command, and
# FETCH_SIZE / WRITE_SIZE in separate --pmc passes, then smoke().  Output under
# gpurun_out/$OUT (default ev).  Stops at the first fault / abort / timeout.
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-ev}
mkdir -p "$O"
fatal() { case "$1" in 0|1) return 1;; *) return 0;; esac; }
step() { local lim=$1 log=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$O/$log" 2>&1
  local rc=$?; echo "[$log] rc=$rc"; tail -${TAILN:-3} "$O/$log" | cut -c1-600
  if fatal $rc || { [ $rc = 1 ] && [ "${STRICT:-1}" = 1 ]; }; then exit $rc; fi; }
[ "${DO_TEST:-1}" != 0 ] && step 900 pytest_gpu.log python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread
[ "${DO_SMOKE:-1}" != 0 ] && step 120 smoke.log python -c "import __graft_entry__ as g; g.smoke()"
[ "${DO_CFG:-1}" != 0 ] && TAILN=2 step 600 bench_configs.log python tools/bench_configs.py
[ "${DO_BENCH:-1}" != 0 ] && step 400 bench.log python bench.py --steps 20 --warmup 5
[ "${DO_BENCH:-1}" != 0 ] && step 400 bench_rep.log python bench.py --steps 40 --warmup 5 --cpu-seconds 0
if [ "${DO_PROF:-1}" != 0 ]; then
  step 400 rocprof_stats.log rocprofv3 --kernel-trace --stats -d "$O/prof" -o bench --output-format csv -- python3 bench.py --steps 20 --warmup 5 --cpu-seconds 0
  step 300 pmc_fetch.log rocprofv3 --pmc FETCH_SIZE -d "$O/pmc_fetch" -o f --output-format csv -- python3 bench.py --steps 12 --warmup 2 --cpu-seconds 0
  step 300 pmc_write.log rocprofv3 --pmc WRITE_SIZE -d "$O/pmc_write" -o w --output-format csv -- python3 bench.py --steps 12 --warmup 2 --cpu-seconds 0
fi
exit 0
