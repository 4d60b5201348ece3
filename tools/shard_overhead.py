"""Per-pivot cost of the sharded pipeline at the config-4 shard shape, on one
GPU: a 1-rank RCCL communicator running prep -> all-gather -> finish -> elim
over rows [0, 1024) of the config-3 tableau, against the single-GPU path on
the same block (norm -> elim).  Run under rocprofv3 for the kernel breakdown.
Prints one JSON line per mode."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "simplex-solver_amd"))

from simplex_amd import dist, synth  # noqa: E402
from simplex_amd.engine import DeviceTableau  # noqa: E402

m, n, rows = 8192, 8192, int(os.environ.get("SHARD_ROWS", "1024"))
T, obj, basis = synth.tableau_rows("dense", m, n, 20251205, 0, rows, order="F")
WINDOWS = [int(x) for x in os.environ.get("SHARD_WINDOWS", "0").split(",")]
for mode, K in [(m_, k_) for k_ in WINDOWS for m_ in ("single", "sharded_rccl1")]:
    if mode == "single":
        eng = DeviceTableau(0)
    else:
        eng = dist.ShardedTableau(0, 0, 1, dist.make_unique_id())
    eng.set_window(K)
    # a 1024-row LP on its own: its own basis entries, objective row shared
    eng.load_rows(T, obj, basis[:rows], rows, 0)
    eng.run_pivots(20)
    eng.sync()
    k = int(os.environ.get("SHARD_PIVOTS", "480"))
    t0 = time.perf_counter()
    eng.run_pivots(k)
    eng.sync()
    el = time.perf_counter() - t0
    st, it, _ = eng.state()
    print(json.dumps({"mode": mode, "window": K, "rows": rows, "cols": n + m + 1, "pivots": k,
                      "us_per_pivot": 1e6 * el / k, "status": st, "iters": it}), flush=True)
    eng.close()
