#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python tools/tune_elim.py > gpurun_out/tune_cfg3.log 2>&1 || exit $?
TUNE_M=1024 TUNE_N=15360 TUNE_PADS=0,64,256 timeout -k 10 600 python tools/tune_elim.py > gpurun_out/tune_m1024.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 400 --cpu-seconds 12 > gpurun_out/bench_default.log 2>&1 || exit $?
tail -1 gpurun_out/bench_default.log | cut -c1-300
