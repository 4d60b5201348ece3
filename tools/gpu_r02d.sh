#!/bin/bash
# chain tests, per-block probe, A/B bench (persistent vs lazy).  Stop at the first fault.
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_chain.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_chain.log 2>&1
rc=$?; echo "pytest chain rc=$rc"; tail -3 gpurun_out/pytest_chain.log; if [ $rc != 0 ]; then exit $rc; fi
timeout -k 10 120 python tools/probe_phases.py --window 24 --chain 0 > gpurun_out/phases_chain0.log 2>&1
rc=$?; echo "probe rc=$rc"; head -12 gpurun_out/phases_chain0.log; grep -A12 per-block gpurun_out/phases_chain0.log; if [ $rc != 0 ]; then exit $rc; fi
for ch in ${CHAINS:-0 1 0 1}; do
  timeout -k 10 200 python bench.py --cpu-seconds 0 --chain $ch > gpurun_out/bench_chain$ch.log 2>&1
  rc=$?; echo "bench chain=$ch rc=$rc"; tail -1 gpurun_out/bench_chain$ch.log | cut -c1-200; if [ $rc != 0 ]; then exit $rc; fi
done
exit 0
