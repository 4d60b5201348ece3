"""Sweep elimination-kernel variants on the config-3 tableau, in one process.

For each column padding (layout, needs a reload) every variant is timed in
interleaved rounds (guide §5.4 rule 24).  One JSON line per (pad, variant):
median/min per-launch time and GB/s on the algorithmic bytes."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "simplex-solver_amd"))
import numpy as np  # noqa: E402

from simplex_amd import synth  # noqa: E402
from simplex_amd.engine import DeviceTableau  # noqa: E402

m = int(os.environ.get("TUNE_M", "8192"))
n = int(os.environ.get("TUNE_N", str(m)))
pads = [int(x) for x in os.environ.get("TUNE_PADS", "256").split(",")]
# (R, grid target, nt flags, interleave bits: 1 = interleaved, +2 = no pipelining)
variants = [(4, 1280, 2, 1), (4, 1280, 2, 5), (4, 1280, 0, 1), (4, 1280, 0, 5),
            (4, 2560, 2, 5), (8, 1280, 2, 5), (4, 1024, 2, 5)]
Tf, obj, basis = synth.tableau_rows("dense", m, n, 20251205, order="F")
print(json.dumps({"m": m, "n": n, "N": n + m + 1}), flush=True)
for pad in pads:
    eng = DeviceTableau(0)
    eng.set_ld_pad(pad)
    eng.load_rows(Tf, obj, basis, m, 0)
    res = {v: [] for v in variants}
    eng.run_pivots(10)
    eng.sync()
    for rnd in range(int(os.environ.get("TUNE_ROUNDS", "3"))):
        for v in variants:
            eng.set_elim_variant(*v)
            eng.elim_timing(reset=True)
            eng.run_pivots(16, time_elim=True, use_graph=False)
            ms, cnt, cols = eng.elim_timing(reset=True)
            res[v].append((ms / cnt, cols / cnt))
    for v in variants:
        t = np.array([a for a, _ in res[v]])
        cols = np.mean([b for _, b in res[v]])
        by = 16.0 * m * (cols - 1) + 8.0 * m
        print(json.dumps({"pad": pad, "R": v[0], "wgs": v[1], "nt": v[2], "ilv": v[3],
                          "us_med": 1e3 * float(np.median(t)), "us_min": 1e3 * float(t.min()),
                          "GBps_med": by / (float(np.median(t)) * 1e-3) / 1e9}), flush=True)
    eng.close()
