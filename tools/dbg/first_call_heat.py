"""Is the slow first timed call (tools/dbg/first_call.py) a GPU-state warm-up
(clocks / power) or a warm-up of this tableau's data? (diagnostic)  Config 3,
K = 24: load, optionally keep the GPU busy on ANOTHER context for ~HEAT_MS
(HEAT=1: a second config-3 tableau's windows, none of the timed context's
data), then 5 warmup windows and the bench's timed call (20 windows,
time_elim = 8) repeated 4 times.
usage: HEAT=0|1 python tools/dbg/first_call_heat.py
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "simplex-solver_amd"))
from simplex_amd import synth  # noqa: E402
from simplex_amd.engine import DeviceTableau  # noqa: E402

K = 24
heat = os.environ.get("HEAT", "0") == "1"
opts = dict(rule="dantzig", skip_zero_cols=True, use_graph=True, chunk=32)
Tf, obj, basis = synth.tableau_rows("dense", 8192, 8192, 20251205, order="F")
e = DeviceTableau(0)
e.set_window(K)
e.load_rows(Tf, obj, basis, 8192, 0)
h = None
if heat:
    h = DeviceTableau(0)
    h.set_window(K)
    Th, oh, bh = synth.tableau_rows("dense", 8192, 8192, 7, order="F")
    h.load_rows(Th, oh, bh, 8192, 0)
    del Th
    h.run_pivots(K, **opts)
    h.sync()
del Tf
if h is not None:
    t0 = time.perf_counter()
    h.run_pivots(40 * K, **opts)  # ~16 ms of the other context's windows
    h.sync()
    print(f"heater: 40 windows of another tableau in {(time.perf_counter() - t0) * 1e3:.1f} ms")
e.run_pivots(5 * K, **opts)
e.sync()
e.elim_timing(reset=True)
for rep in range(4):
    e.sync()
    t0 = time.perf_counter()
    e.run_pivots(20 * K, time_elim=8, **opts)
    e.sync()
    dt = time.perf_counter() - t0
    ms, n, _ = e.elim_timing(reset=True)
    print(f"heat {int(heat)}: call {rep}: {dt * 1e3:.3f} ms = {20 * K / dt:.0f} pivots/s, "
          f"flush {ms / max(n, 1) * 1e3:.1f} us (events, {n} launches)")
e.close()
if h is not None:
    h.close()
