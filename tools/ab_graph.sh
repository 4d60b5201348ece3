#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { local tag=$1; shift
  timeout -k 10 300 python bench.py --steps 400 --cpu-seconds 0 "$@" > gpurun_out/ab_$tag.log 2>&1 || exit $?
  tail -1 gpurun_out/ab_$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$tag', round(d['value']), round(d['ms_per_step']*1e3,1), round(r['avg_launch_us'],1), round(r['frac'],3), d['config']['elim_variant'])"
}
run default
run pipe1 --ilv 1
run pipe0 --ilv 3
run pipe1nt0 --ilv 1 --nt 0
run default_again
timeout -k 10 900 python -m pytest tests -m gpu -q > gpurun_out/pytest_all.log 2>&1; echo "pytest rc=$?"; tail -3 gpurun_out/pytest_all.log
