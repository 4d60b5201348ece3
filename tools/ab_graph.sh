#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { local tag=$1; shift
  timeout -k 10 300 python bench.py --steps 400 --cpu-seconds 0 "$@" > gpurun_out/ab_$tag.log 2>&1 || exit $?
  tail -1 gpurun_out/ab_$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$tag', round(d['value']), round(d['ms_per_step']*1e3,1), round(r['avg_launch_us'],1), round(r['frac'],3))"
}
run g1e8 --graph 1 --time-every 8
run g0e1 --graph 0 --time-every 1
run g1e1 --graph 1 --time-every 1
run g0e8 --graph 0 --time-every 8
run g1e8_expl --graph 1 --time-every 8 --nt 2 --ilv 3 --R 4 --wgs 1280 --ld-pad 256
TUNE_M=2048 TUNE_N=14336 TUNE_PADS=0,64,256 timeout -k 10 600 python tools/tune_elim.py > gpurun_out/tune_m2048.log 2>&1 || exit $?
TUNE_M=4096 TUNE_N=12288 TUNE_PADS=0,64,256 timeout -k 10 600 python tools/tune_elim.py > gpurun_out/tune_m4096.log 2>&1 || exit $?
