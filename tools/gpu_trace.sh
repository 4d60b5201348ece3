#!/bin/bash
# Kernel trace of the bench (gaps between a window's launches: tools/trace_gaps.py)
# and the full-solve timings of configs 3 and 5 (tools/bench_configs.py --full).
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-trace}; mkdir -p $O
fatal() { case "$1" in 0|1) return 1;; *) return 0;; esac; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o bench --output-format csv -- python3 bench.py --cpu-seconds 0 ${BENCH_ARGS:-} > $O/rocprof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; grep '^{' $O/rocprof.log | cut -c1-300; if fatal $rc; then exit $rc; fi
if [ "${FULL:-1}" != 0 ]; then
  timeout -k 10 300 python tools/bench_configs.py --full > $O/full.log 2>&1
  rc=$?; echo "full rc=$rc"; cut -c1-400 $O/full.log; if fatal $rc; then exit $rc; fi
fi
exit 0
