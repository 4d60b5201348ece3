#!/bin/bash
# Round-3 measurements: shard overhead (peer chain vs RCCL at the config-4
# shard shape), the driver's bench command, its rocprofv3 kernel stats, SQ /
# GRBM counters of the K = 24 and K = 32 flush, a K = 32 bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r03e}
mkdir -p $O
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $O/$name.log 2>&1
  local rc=$?; echo "[$name] rc=$rc"; tail -3 $O/$name.log | cut -c1-400
  case $rc in 0) ;; *) exit $rc;; esac
}
run shard 240 python tools/shard_overhead.py
run bench 300 python bench.py --steps 20 --warmup 5
run prof 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --cpu-seconds 0
for K in 24 32; do
  run pmc_k$K 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT -d $O/pmc_k$K -o p --output-format csv -- python3 bench.py --steps 16 --warmup 4 --cpu-seconds 0 --window $K
done
run bench_k32 300 python bench.py --steps 20 --warmup 5 --window 32 --cpu-seconds 0
exit 0
