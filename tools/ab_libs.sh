#!/bin/bash
# Same-box A/B of library variants and environment settings on the bench
# (round 6).  VARIANTS: label=lib[=VAR=value] ... (lib under
# simplex-solver_amd/simplex_amd/lib); ROUNDS; ABSTEPS; OUT; TAG.
set -u
cd "${GRAFT_REPO_ROOT}"; export TMPDIR=/tmp
O=gpurun_out/${OUT:-r06}; mkdir -p $O
J=$O/ab${TAG:-}.jsonl
for r in ${ROUNDS:-1 2}; do for v in $VARIANTS; do
  lab=${v%%=*}; rest=${v#*=}; lib=${rest%%=*}; asg=""; [ "$rest" != "$lib" ] && asg=${rest#*=}
  log=$O/ab${TAG:-}_${lab}_r$r.log
  env $asg SPX_LIB=$PWD/simplex-solver_amd/simplex_amd/lib/$lib SPX_LIB_PARTIAL=1 \
    timeout -k 10 300 python bench.py --steps ${ABSTEPS:-40} --warmup 5 --cpu-seconds 0 > $log 2>&1
  rc=$?; [ $rc != 0 ] && { echo "[$lab r$r] rc=$rc"; tail -5 $log; exit $rc; }
  python - "$log" "$lab" "$r" >> $J <<'PY'
import json, sys
l = [x for x in open(sys.argv[1]) if x.startswith("{")][-1]
d = json.loads(l)
print(json.dumps({"variant": sys.argv[2], "round": int(sys.argv[3]), "value": round(d["value"], 1),
                  "ms_per_step": round(d["ms_per_step"], 4), "flush_us": round(d["roofline"]["avg_launch_us"], 1),
                  "frac": round(d["roofline"]["frac"], 4),
                  "chain_us_per_pivot": round(d["chain"]["us_per_pivot"], 3)}))
PY
  tail -1 $J
done; done
