#!/bin/bash
# Persistent-chain first run: its parity tests, the window suite, smoke, then
# an A/B bench (persistent chain vs launch per phase).  Stop at the first fault.
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
fatal() { case "$1" in 0|1) return 1;; *) return 0;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_chain.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_chain.log 2>&1
rc=$?; echo "pytest chain rc=$rc"; tail -15 gpurun_out/pytest_chain.log; if [ $rc != 0 ]; then exit $rc; fi
timeout -k 10 400 python -u -m pytest tests/test_gpu_window.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_window.log 2>&1
rc=$?; echo "pytest window rc=$rc"; tail -4 gpurun_out/pytest_window.log; if [ $rc != 0 ]; then exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log; if [ $rc != 0 ]; then exit $rc; fi
for ch in 0 1 0 1; do
  timeout -k 10 200 python bench.py --cpu-seconds 0 --chain $ch > gpurun_out/bench_chain$ch.log 2>&1
  rc=$?; echo "bench chain=$ch rc=$rc"; tail -1 gpurun_out/bench_chain$ch.log | cut -c1-200; if [ $rc != 0 ]; then exit $rc; fi
done
exit 0
