#!/bin/bash
# Phase timestamps of one window (probe build): persistent chain vs lazy kernels.
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
for ch in ${CHAINS:-0 1}; do
  timeout -k 10 120 python tools/probe_phases.py --window ${K:-24} --chain $ch > gpurun_out/phases_chain$ch.log 2>&1
  rc=$?; echo "probe chain=$ch rc=$rc"; head -${LINES_SHOW:-50} gpurun_out/phases_chain$ch.log; if [ $rc != 0 ]; then exit $rc; fi
done
exit 0
