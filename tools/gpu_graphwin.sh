#!/bin/bash
# Windows per replayed graph: parity suites, then a same-box A/B of
# SPX_GRAPH_WINDOWS=4 (default) against 1 (one graph per window, round 2-3),
# the bench and the config-2 / config-5 timings.
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-gw}; mkdir -p $O
fatal() { case "$1" in 0|1) return 1;; *) return 0;; esac; }
timeout -k 10 900 python -u -m pytest ${TESTS:-tests/test_gpu_window.py tests/test_gpu_chain.py tests/test_gpu_engine.py} -m gpu -x -q \
  --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc != 0 ] && { grep -B5 -A40 "Error\|FAIL" $O/pytest.log | head -80; exit $rc; }
OUT=${OUT:-gw} ROUNDS=${ROUNDS:-3} CONFIGS="${CONFIGS:-env:SPX_GRAPH_WINDOWS=4|--window 24;env:SPX_GRAPH_WINDOWS=1|--window 24}" bash tools/gpu_sweep.sh || exit $?
for gw in 4 1; do
  SPX_GRAPH_WINDOWS=$gw timeout -k 10 400 python tools/bench_configs.py > $O/configs_gw$gw.log 2>&1
  rc=$?; echo "configs gw=$gw rc=$rc"; cut -c1-200 $O/configs_gw$gw.log; if fatal $rc; then exit $rc; fi
done
exit 0
