# column-padding A/B on configs 5 and the full solves (tools/bench_configs.py, SPX_LD_PAD)
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/pad_configs.jsonl
: > $out
for r in 0 1 2; do
  for p in 256 1024; do
    SPX_LD_PAD=$p timeout -k 10 150 python tools/bench_configs.py --config5-k24 >> $out || exit 1
    SPX_LD_PAD=$p timeout -k 10 200 python tools/bench_configs.py --full >> $out || exit 1
    tail -3 $out | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['config'][:40], 'pad', d['ld_pad'], round(d['gpu_pivots_per_s']), d.get('matches_fixture', d.get('first_pivots_match_oracle')), flush=True)"
  done
done
