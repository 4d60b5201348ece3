#!/bin/bash
# Round-2 first box run: exchange-latency probe, the driver's bench command,
# the default bench, then the GPU parity suite.  Each step time-limited; stop
# at the first fault.
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
fatal() { case "$1" in 0|1) return 1;; *) return 0;; esac; }
timeout -k 10 120 ./tools/chain_probe > gpurun_out/chain_probe.log 2>&1
rc=$?; echo "probe rc=$rc"; cat gpurun_out/chain_probe.log; if [ $rc != 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver_args.log 2>&1
rc=$?; echo "bench(driver args) rc=$rc"; tail -1 gpurun_out/bench_driver_args.log | cut -c1-300; if fatal $rc; then exit $rc; fi
timeout -k 10 300 python bench.py --cpu-seconds 0 > gpurun_out/bench_default.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_default.log | cut -c1-300; if fatal $rc; then exit $rc; fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_all.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_all.log
exit $rc
