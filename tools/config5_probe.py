"""How long is Bland's path on config 5?  Solves the degenerate 4096 x 4096
LP (synth 'degenerate', seed 5) on one GPU at K = 24 in chunks until optimal
or the time budget, printing the pivot count, status and objective."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "simplex-solver_amd"))
from simplex_amd import synth  # noqa: E402
from simplex_amd.engine import DeviceTableau  # noqa: E402

budget = float(os.environ.get("PROBE_SECONDS", "90"))
T, basis = synth.full_tableau("degenerate", 4096, 4096, 5)
with DeviceTableau(0) as e:
    e.set_window(24)
    e.load(T, basis)
    del T
    t0 = time.perf_counter()
    while True:
        r = e.solve(rule="bland", max_iters=1 << 20)
        st, it, z = e.state()
        el = time.perf_counter() - t0
        print(json.dumps({"pivots": it, "status": r.status, "z": z, "seconds": el,
                          "pivots_per_s": it / el}), flush=True)
        if r.status != 1 or el > budget:
            break
