#!/bin/bash
# Round evidence: full parity suite, config 2/5 timings, bench (with CPU
# baseline; and the driver's command), the shard-overhead modes, rocprofv3 kernel trace + stats of the same bench command, and
# FETCH_SIZE / WRITE_SIZE in separate --pmc passes.  Stops at the first fault.
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out/final
fatal() { case "$1" in 0|1) return 1;; *) return 0;; esac; }
step() { local lim=$1 log=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/final/$log" 2>&1
  local rc=$?; echo "[$log] rc=$rc"; tail -${TAILN:-3} "gpurun_out/final/$log" | cut -c1-400
  if fatal $rc; then exit $rc; fi; }
[ "${DO_TEST:-1}" != 0 ] && step 900 pytest_gpu.log python -m pytest tests -m gpu -q
[ "${DO_CFG:-1}" != 0 ] && TAILN=2 step 600 bench_configs.log python tools/bench_configs.py
step 400 bench.log python bench.py --cpu-seconds 15
step 400 bench_driver.log python bench.py --steps 20 --warmup 5
[ "${DO_SHARD:-1}" != 0 ] && step 300 shard.log python tools/shard_overhead.py
step 400 rocprof_stats.log rocprofv3 --kernel-trace --stats -d gpurun_out/final/prof -o bench --output-format csv -- python3 bench.py --cpu-seconds 0
step 400 pmc_fetch.log rocprofv3 --pmc FETCH_SIZE -d gpurun_out/final/pmc_fetch -o f --output-format csv -- python3 bench.py --steps 128 --warmup 16 --cpu-seconds 0
step 400 pmc_write.log rocprofv3 --pmc WRITE_SIZE -d gpurun_out/final/pmc_write -o w --output-format csv -- python3 bench.py --steps 128 --warmup 16 --cpu-seconds 0

step 120 smoke.log python -c "import __graft_entry__ as g; g.smoke()"
exit 0
