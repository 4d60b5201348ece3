"""Is the bench's single timed call slower than later identical calls?
(diagnostic)  Config 3, K = 24: load, 5 warmup windows (as bench.py
--warmup 5), then the bench's timed call (20 windows, time_elim = 8) repeated
8 times back to back, each timed by wall clock around call + sync.
usage: python tools/dbg/first_call.py [warmup_windows]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "simplex-solver_amd"))
from simplex_amd import synth  # noqa: E402
from simplex_amd.engine import DeviceTableau  # noqa: E402

K = 24
W = int(sys.argv[1]) if len(sys.argv) > 1 else 5
Tf, obj, basis = synth.tableau_rows("dense", 8192, 8192, 20251205, order="F")
e = DeviceTableau(0)
e.set_window(K)
e.load_rows(Tf, obj, basis, 8192, 0)
del Tf
opts = dict(rule="dantzig", skip_zero_cols=True, use_graph=True, chunk=32)
e.run_pivots(W * K, **opts)
e.sync()
e.elim_timing(reset=True)
for rep in range(8):
    e.sync()
    t0 = time.perf_counter()
    e.run_pivots(20 * K, time_elim=8, **opts)
    e.sync()
    dt = time.perf_counter() - t0
    ms, n, _ = e.elim_timing(reset=True)
    print(f"warmup {W}: call {rep}: {dt * 1e3:.3f} ms = {20 * K / dt:.0f} pivots/s, "
          f"flush {ms / max(n, 1) * 1e3:.1f} us (events, {n} launches)")
e.close()
