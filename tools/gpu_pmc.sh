#!/bin/bash
# PMC passes (one counter group each, kernel-trace only) over a short bench run.
# usage: PMC_ARGS="bench args" bash tools/gpu_pmc.sh "SQ_A SQ_B ..." "SQ_C ..." ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
n=0
for grp in "$@"; do
  n=$((n+1))
  timeout -k 10 300 rocprofv3 --pmc $grp -d gpurun_out/pmc/p$n -o p --output-format csv -- python3 bench.py --steps 64 --warmup 16 --cpu-seconds 0 ${PMC_ARGS:-} > gpurun_out/pmc/p$n.log 2>&1
  rc=$?; echo "[pmc $n: $grp] rc=$rc"; tail -2 gpurun_out/pmc/p$n.log | cut -c1-300
  case $rc in 0|1) ;; *) exit $rc;; esac
done
exit 0
