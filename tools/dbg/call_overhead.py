"""Per-call fixed overhead of spx_run_pivots at config 3 (diagnostic).

Times wall-clock run_pivots(n) + sync for several window counts n (the
bench's timed region shape, time_elim = 8) and fits t = a + b n: a is the
fixed cost of one call (begin_call, admission, the release callback, ...).
Also times the host side of the call alone (enqueue) and a bare sync.
usage: python tools/dbg/call_overhead.py
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "simplex-solver_amd"))
from simplex_amd import synth  # noqa: E402
from simplex_amd.engine import DeviceTableau  # noqa: E402

K = 24
Tf, obj, basis = synth.tableau_rows("dense", 8192, 8192, 20251205, order="F")
e = DeviceTableau(0)
e.set_window(K)
e.load_rows(Tf, obj, basis, 8192, 0)
del Tf
opts = dict(rule="dantzig", skip_zero_cols=True, use_graph=True, chunk=32)
e.run_pivots(5 * K, **opts)
e.sync()
label = os.environ.get("LABEL", "default")
rows = []
for rep in range(3):
    for nw in (1, 2, 5, 10, 20, 40):
        e.sync()
        t0 = time.perf_counter()
        e.run_pivots(nw * K, time_elim=8, **opts)
        t1 = time.perf_counter()
        e.sync()
        t2 = time.perf_counter()
        rows.append((nw, (t2 - t0) * 1e3, (t1 - t0) * 1e3))
        e.elim_timing(reset=True)
t0 = time.perf_counter()
for _ in range(20):
    e.sync()
bare = (time.perf_counter() - t0) / 20 * 1e3
nws = np.array([r[0] for r in rows], float)
ts = np.array([r[1] for r in rows], float)
b, a = np.polyfit(nws, ts, 1)
print(f"[{label}] fit: {a * 1e3:.1f} us per call + {b * 1e3:.1f} us per window; bare sync {bare * 1e3:.1f} us")
for nw in (1, 2, 5, 10, 20, 40):
    sel = [r for r in rows if r[0] == nw]
    print(f"[{label}] windows {nw:3d}: wall {min(r[1] for r in sel):8.3f} ms (best of 3), "
          f"host enqueue {min(r[2] for r in sel):7.3f} ms")
e.close()
