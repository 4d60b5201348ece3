#!/bin/bash
# A/B of the timed-region event sampling and a plain bench line
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for k in 1 8 64; do
  timeout -k 10 300 python bench.py --steps 400 --cpu-seconds 0 --time-every $k > gpurun_out/ab_every$k.log 2>&1 || exit $?
  tail -1 gpurun_out/ab_every$k.log | cut -c1-400
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof8 -o bench --output-format csv -- python3 bench.py --steps 200 --cpu-seconds 0 --time-every 8 > gpurun_out/prof8.log 2>&1 || exit $?
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_all.log 2>&1; echo "pytest rc=$?"; tail -3 gpurun_out/pytest_all.log
