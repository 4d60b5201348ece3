#!/bin/bash
# chain + window parity tests, phase probe (fine stamps), bench repeats.  Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT}"; export TMPDIR=/tmp; O=gpurun_out/${OUT:-ch}; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_chain.py ${TESTS:-} -x -q --timeout 120 --timeout-method thread > $O/pytest_chain.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_chain.log; [ $rc != 0 ] && exit $rc
timeout -k 10 120 python tools/probe_phases.py --window 24 > $O/phases24.log 2>&1
rc=$?; echo "probe rc=$rc"; head -${PHN:-20} $O/phases24.log; [ $rc != 0 ] && exit $rc
OUT=${OUT:-ch} ROUNDS=${ROUNDS:-2} CONFIGS="${CONFIGS:---window 24}" bash tools/gpu_sweep.sh
