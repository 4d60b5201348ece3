"""pivots/s of K=16 windows on config 3: direct launches vs per-window graph
replays vs one graph of all windows (no events)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "simplex-solver_amd"))
from simplex_amd import synth
from simplex_amd.engine import DeviceTableau
m = n = 8192
Tf, obj, basis = synth.tableau_rows("dense", m, n, 20251205, order="F")
e = DeviceTableau(0); e.set_window(16); e.load_rows(Tf, obj, basis, m, 0); del Tf
e.run_pivots(64); e.sync()
for rnd in range(2):
    for mode in ("direct", "graph/window", "graph/all(timed,every 1000)"):
        S = 512
        kw = dict(use_graph=(mode != "direct"))
        if mode.startswith("graph/all"):
            e.run_pivots(S, time_elim=1000, **kw); e.sync()  # build + warm
        t0 = time.perf_counter()
        if mode.startswith("graph/all"):
            e.run_pivots(S, time_elim=1000, **kw)
        else:
            e.run_pivots(S, **kw)
        e.sync()
        el = time.perf_counter() - t0
        print(f"{rnd} {mode:28s} {S / el:9.0f} pivots/s", flush=True)
e.close()
