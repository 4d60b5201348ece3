set -u
cd "${GRAFT_REPO_ROOT}"; export TMPDIR=/tmp; mkdir -p gpurun_out/dyn1
timeout -k 10 400 python -u -m pytest tests/test_gpu_window.py -x -q --timeout 120 --timeout-method thread > gpurun_out/dyn1/pytest_window.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/dyn1/pytest_window.log; [ $rc != 0 ] && exit $rc
timeout -k 10 120 env PROBE_NPZ=gpurun_out/dyn1/flush24dyn.npz python tools/probe_phases.py --window 24 --fv 32 > gpurun_out/dyn1/phases24dyn.log 2>&1
rc=$?; echo "probe rc=$rc"; tail -14 gpurun_out/dyn1/phases24dyn.log; [ $rc != 0 ] && exit $rc
OUT=dyn1 ROUNDS=3 CONFIGS="--window 24;--window 24 --fv 32;--window 32 --fv 32" bash tools/gpu_sweep.sh
