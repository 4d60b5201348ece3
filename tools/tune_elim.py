"""Sweep elimination-kernel variants in ONE process on the config-3 tableau
(interleaved rounds, guide §5.4 rule 24).  Prints one JSON line per variant
with the median/min per-launch time and GB/s on the algorithmic bytes."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "simplex-solver_amd"))
import numpy as np  # noqa: E402

from simplex_amd import synth  # noqa: E402
from simplex_amd.engine import DeviceTableau  # noqa: E402

m = n = int(os.environ.get("TUNE_M", "8192"))
variants = [(R, wgs, nt, ilv) for R in (4, 8) for wgs in (1280, 2048, 4096, 8192)
            for nt in (0, 2) for ilv in (0, 1)]
Tf, obj, basis = synth.tableau_rows("dense", m, n, 20251205, order="F")
eng = DeviceTableau(0)
eng.load_rows(Tf, obj, basis, m, 0)
del Tf
res = {v: [] for v in variants}
eng.run_pivots(10)
eng.sync()
for rnd in range(int(os.environ.get("TUNE_ROUNDS", "4"))):
    for v in variants:
        R, wgs, nt, ilv = v
        eng.set_elim_variant(R, wgs, nt, ilv)
        eng.elim_timing(reset=True)
        eng.run_pivots(24, time_elim=True)
        ms, cnt, cols = eng.elim_timing(reset=True)
        res[v].append((ms / cnt, cols / cnt))
for v in variants:
    t = np.array([a for a, _ in res[v]])
    cols = np.mean([b for _, b in res[v]])
    by = 16.0 * m * (cols - 1) + 8.0 * m
    print(json.dumps({"R": v[0], "wgs": v[1], "nt": v[2], "ilv": v[3], "us_med": 1e3 * float(np.median(t)),
                      "us_min": 1e3 * float(t.min()),
                      "GBps_med": by / (float(np.median(t)) * 1e-3) / 1e9}), flush=True)
eng.close()
