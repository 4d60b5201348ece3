set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/${OUT:-pad_sweep}.jsonl
: > $out
for r in ${ROUNDS:-0 1}; do
  for p in ${PADS:-256 0 64 128 192 320 512 1024 2048}; do
    line=$(timeout -k 10 150 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 --ld-pad $p 2>gpurun_out/pad_err.log | tail -1) || { echo "pad $p failed"; cat gpurun_out/pad_err.log | tail -20; exit 1; }
    echo "{\"round\": $r, \"ld_pad\": $p, \"bench\": $line}" >> $out
    python - "$line" "$p" <<'PY'
import json,sys
d=json.loads(sys.argv[1]); 
def f(k,o=d):
    return o.get(k)
ch=d.get("chain",{}); fl=d.get("roofline",{})
print("pad", sys.argv[2], "pivots/s", round(d["value"]), "chain us/piv", ch.get("us_per_pivot"), "flush frac", fl.get("frac"), flush=True)
PY
  done
done
