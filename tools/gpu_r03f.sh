#!/bin/bash
# Round-3 row_fix beside the flush: the window / chain / engine / full-size
# parity suites, then a same-box A/B: this tree with row_fix on a side stream
# (default), the same with SPX_ROWFIX_BESIDE=0, and the previous library (pre).
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-fix}; mkdir -p $O
timeout -k 10 900 python -u -m pytest ${TESTS:-tests/test_gpu_window.py tests/test_gpu_chain.py tests/test_gpu_fullsize.py} -m gpu -x -q \
  --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc != 0 ] && { grep -B5 -A40 "Error\|FAIL" $O/pytest.log | head -80; exit $rc; }
OUT=${OUT:-fix} ROUNDS=${ROUNDS:-3} CONFIGS="${CONFIGS:---window 24;env:SPX_ROWFIX_BESIDE=0|--window 24;pre|--window 24;--window 32;pre|--window 32}" bash tools/gpu_sweep.sh
