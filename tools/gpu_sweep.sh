#!/bin/bash
# A/B sweep of bench.py configurations, interleaved over ROUNDS rounds, one
# bench process per configuration.  CONFIGS: ';'-separated bench argument
# lists, each optionally prefixed "NAME|" to run with
# simplex_amd/lib/libspx_NAME.so (same-box A/B of two builds) or, as
# "env:VAR=VALUE|", with that environment variable set.  Output:
# gpurun_out/$OUT/sweep.jsonl (value + flush time per run).
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-sweep}
mkdir -p "$O"
IFS=';' read -ra CF <<< "${CONFIGS}"
for r in $(seq 1 "${ROUNDS:-2}"); do
  for cfg in "${CF[@]}"; do
    lib=""; c="$cfg"; envs=""
    if [[ "$cfg" == *"|"* ]]; then lib="${cfg%%|*}"; c="${cfg#*|}"; fi
    # "env:VAR=VALUE|args": run with that environment variable instead of another library
    if [[ "$lib" == env:* ]]; then envs="${lib#env:}"; lib=""; fi
    if [ -n "$lib" ]; then export SPX_LIB="$PWD/simplex-solver_amd/simplex_amd/lib/libspx_$lib.so" SPX_LIB_PARTIAL=1; else unset SPX_LIB SPX_LIB_PARTIAL; fi
    env $envs timeout -k 10 200 python bench.py --cpu-seconds 0 ${STEPS:---steps 40 --warmup 5} $c > "$O/last.log" 2>&1
    rc=$?
    if [ $rc != 0 ]; then echo "config [$c] rc=$rc"; tail -5 "$O/last.log"; exit $rc; fi
    python - "$cfg" "$r" "$O/last.log" >> "$O/sweep.jsonl" <<'EOF'
import json, sys
d = json.loads([l for l in open(sys.argv[3]) if l.startswith("{")][-1])
print(json.dumps({"args": sys.argv[1], "round": int(sys.argv[2]), "value": round(d["value"], 1),
                  "ms_per_step": round(d["ms_per_step"], 4), "flush_us": round(d["roofline"]["avg_launch_us"], 1),
                  "frac": round(d["roofline"]["frac"], 4), "chain_blocks": d["config"].get("chain_blocks"),
                  "chain_us_per_pivot": round((d.get("chain") or {}).get("us_per_pivot", 0), 3),
                  "groups": d["config"]["elim_variant"].get("flush_groups")}))
EOF
    tail -1 "$O/sweep.jsonl"
  done
done
exit 0
