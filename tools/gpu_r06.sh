#!/bin/bash
# Round-6 GPU steps: STEPS="probe tests bench ..." (each under its own time
# limit; stops at the first failure, GPU fault or time limit).
set -u
cd "${GRAFT_REPO_ROOT}"; export TMPDIR=/tmp
O=gpurun_out/${OUT:-r06}; mkdir -p $O
run() { local lim=$1 log=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$O/$log" 2>&1
  local rc=$?; echo "[$log] rc=$rc"; tail -${TAILN:-4} "$O/$log" | cut -c1-600
  [ $rc != 0 ] && exit $rc; return 0; }
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
for s in ${STEPS:-probe tests bench}; do
  case $s in
    ipcdiag) # the IPC reload diagnostic: addresses, handles, mapped peers per
        # load; no pivots run.  IPCENV e.g. "SPX_IPC_ORDER=0" (round 4 order, no keep)
        TAILN=20 run 240 ipcdiag${PHTAG:-}.log env ${IPCENV:-SPX_IPC_KEEP=0} python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 --master-port 29541 tools/rccl_ranks_check.py --peer 2 --same-device --rows 512 --cols 2048 --window 24 --then 1024x8000,512x2048,1024x8000,512x2048 --ipc-log --no-solve ;;
    same8) TAILN=2 run 500 bench_same8.log python -m torch.distributed.run --nnodes=1 --nproc-per-node=8 --master-addr 127.0.0.1 --master-port 29535 bench.py --gpus 8 --same-device --chain 3 --steps 10 --warmup 2 --cpu-seconds 0 ;;
    sameab) # 2 ranks on GPU 0: the row transports (and the slot chains: SAMEVARS label:row:lean)
        for r in ${ROUNDS:-1 2 3}; do for v in ${SAMEVARS:-pull:pull:1 push:push:1}; do
          lab=${v%%:*}; rest=${v#*:}; row=${rest%%:*}; ln=${rest#*:}
          SPX_CHAIN_LEAN=$ln TAILN=0 run 400 sameab_${lab}_r$r.log python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 --master-port 2954$r bench.py --gpus 2 --same-device --peer-row $row --steps 40 --warmup 5 --cpu-seconds 0
          python - "$O/sameab_${lab}_r$r.log" "$lab" "$r" >> $O/sameab.jsonl <<'PY'
import json, sys
l = [x for x in open(sys.argv[1]) if x.startswith("{")][-1]
d = json.loads(l)
print(json.dumps({"variant": sys.argv[2], "round": int(sys.argv[3]), "value": round(d["value"], 1),
                  "ms_per_step": round(d["ms_per_step"], 4), "flush_us": round(d["roofline"]["avg_launch_us"], 1),
                  "chain_us_per_pivot": round(d["chain"]["us_per_pivot"], 3),
                  "row_transport": d["config"]["peer_chain"].get("row_transport")}))
PY
        done; done; cat $O/sameab.jsonl ;;
    tailsweep) # the flush's tail share (SPX_FLUSH_TAIL %, SPX_FLUSH_TAIL_R0): TAILVARS tail:r0 ...
        for r in ${ROUNDS:-1 2 3}; do for v in ${TAILVARS:-12:0 6:1 9:1 12:1}; do
          tl=${v%%:*}; t0=${v#*:}
          SPX_FLUSH_TAIL=$tl TAILN=0 run 300 tail_${tl}_${t0}_r$r.log python bench.py --steps 40 --warmup 5 --time-every 2 --cpu-seconds 0
          python - "$O/tail_${tl}_${t0}_r$r.log" "$tl:$t0" "$r" >> $O/tailsweep.jsonl <<'PY'
import json, sys
l = [x for x in open(sys.argv[1]) if x.startswith("{")][-1]
d = json.loads(l)
print(json.dumps({"variant": sys.argv[2], "round": int(sys.argv[3]), "value": round(d["value"], 1),
                  "flush_us": round(d["roofline"]["avg_launch_us"], 1), "frac": round(d["roofline"]["frac"], 4),
                  "chain_us_per_pivot": round(d["chain"]["us_per_pivot"], 3)}))
PY
        done; done; cat $O/tailsweep.jsonl ;;
    strag) TAILN=80 run 300 stragglers${PHTAG:-}.log python tools/probe_stragglers.py --windows ${SWIN:-40} --npz $O/stragglers${PHTAG:-}.npz ${PHARGS:-} ;;
    tests) if [ -n "${KEXPR:-}" ]; then
             run 900 pytest_${TTAG:-sel}.log $PYT ${TESTS:-tests/test_gpu_chain.py tests/test_gpu_peer_chain.py} -k "$KEXPR"
           else
             run 900 pytest_${TTAG:-sel}.log $PYT ${TESTS:-tests/test_gpu_chain.py tests/test_gpu_peer_chain.py}
           fi ;;
    suite) run 1100 pytest_gpu.log $PYT -m gpu tests ;;
    userpath) SPX_USER_PATH_JSON=$O/user_path.json TAILN=40 run 900 pytest_user_path.log python -u -m pytest -x -v -s --timeout 700 --timeout-method thread tests/test_gpu_user_path.py ;;
    benchdrv) TAILN=1 run 400 bench_driver_cpu.log python bench.py --steps 20 --warmup 5 ;;
    bench) TAILN=1 run 300 bench_driver.log python bench.py --steps 20 --warmup 5 --cpu-seconds 0 ;;
    bench40) TAILN=1 run 300 bench40.log python bench.py --steps 40 --warmup 5 --cpu-seconds 0 ;;
    benchcpu) TAILN=1 run 400 bench_cpu.log python bench.py --cpu-seconds 15 ;;
    same) TAILN=1 run 400 bench_same.log python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --same-device --steps 20 --warmup 5 --cpu-seconds 0 ;;
    phases) TAILN=30 run 200 phases24${PHTAG:-}.log python tools/probe_phases.py --window 24 ${PHARGS:-} ;;
    smoke) run 200 smoke.log python -c "import __graft_entry__ as g; g.smoke()" ;;
    rocprof) run 400 rocprof.log rocprofv3 --kernel-trace --stats -d $O/prof -o bench --output-format csv -- python3 bench.py --steps 20 --warmup 5 --cpu-seconds 0 ;;
    pmcf|pmcw) c=FETCH_SIZE; [ $s = pmcw ] && c=WRITE_SIZE
        run 300 $s.log rocprofv3 --kernel-trace --pmc $c -d $O/$s -o p --output-format csv -- python3 bench.py --steps 20 --warmup 5 --cpu-seconds 0 ;;
    ab) # VARIANTS: label=lib:chain[:lean] ... (lib relative to simplex-solver_amd/simplex_amd/lib)
        for r in ${ROUNDS:-1 2 3}; do for v in ${VARIANTS:-base=libspx.so:0:0 lean=libspx.so:0:1}; do
          lab=${v%%=*}; rest=${v#*=}; lib=${rest%%:*}; rest=${rest#*:}; c=${rest%%:*}; ln=1; pf=0
          [ "$rest" != "$c" ] && { rest=${rest#*:}; ln=${rest%%:*}; [ "$rest" != "$ln" ] && pf=${rest#*:}; }
          SPX_CHAIN_PF=$pf SPX_CHAIN_LEAN=$ln SPX_LIB=$PWD/simplex-solver_amd/simplex_amd/lib/$lib SPX_LIB_PARTIAL=1 TAILN=0 \
            run 300 ab_${lab}_r$r.log python bench.py --chain $c --steps ${ABSTEPS:-40} --warmup 5 --cpu-seconds 0 ${ABARGS:-}
          python - "$O/ab_${lab}_r$r.log" "$lab" "$r" >> $O/ab.jsonl <<'PY'
import json, sys
l = [x for x in open(sys.argv[1]) if x.startswith("{")][-1]
d = json.loads(l)
print(json.dumps({"variant": sys.argv[2], "round": int(sys.argv[3]), "value": round(d["value"], 1),
                  "ms_per_step": round(d["ms_per_step"], 4), "flush_us": round(d["roofline"]["avg_launch_us"], 1),
                  "frac": round(d["roofline"]["frac"], 4), "chain_blocks": d["config"]["chain_blocks"],
                  "chain_us_per_pivot": round(d["chain"]["us_per_pivot"], 3)}))
PY
        done; done; cat $O/ab.jsonl ;;
    envab) # ENVVARS: label=VAR=value ... (one environment assignment per variant)
        for r in ${ROUNDS:-1 2 3}; do for v in ${ENVVARS:-t12=SPX_FLUSH_TAIL=12 t10=SPX_FLUSH_TAIL=10}; do
          lab=${v%%=*}; asg=${v#*=}
          TAILN=0 run 300 envab_${lab}_r$r.log env $asg python bench.py --steps ${ABSTEPS:-40} --warmup 5 --cpu-seconds 0 ${ABARGS:-}
          python - "$O/envab_${lab}_r$r.log" "$lab" "$r" >> $O/envab${EABTAG:-}.jsonl <<'PY'
import json, sys
l = [x for x in open(sys.argv[1]) if x.startswith("{")][-1]
d = json.loads(l)
print(json.dumps({"variant": sys.argv[2], "round": int(sys.argv[3]), "value": round(d["value"], 1),
                  "ms_per_step": round(d["ms_per_step"], 4), "flush_us": round(d["roofline"]["avg_launch_us"], 1),
                  "frac": round(d["roofline"]["frac"], 4),
                  "chain_us_per_pivot": round(d["chain"]["us_per_pivot"], 3)}))
PY
        done; done; cat $O/envab${EABTAG:-}.jsonl ;;
    rpenv) # rocprof kernel stats under one environment assignment (RPENV, RPTAG)
        run 400 rocprof_${RPTAG:-env}.log env ${RPENV:-SPX_FLUSH_TAIL=12} rocprofv3 --kernel-trace --stats -d $O/prof_${RPTAG:-env} -o bench --output-format csv -- python3 bench.py --steps 20 --warmup 5 --cpu-seconds 0 ;;
    *) echo "unknown step $s"; exit 3 ;;
  esac
done
exit 0
