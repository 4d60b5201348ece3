import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "simplex-solver_amd")); sys.path.insert(0, ROOT)
import numpy as np
from simplex_amd import synth
from simplex_amd.engine import DeviceTableau
T, basis = synth.full_tableau("dense", 64, 96, 7)
for K in (4, 8):
  for lims in [(5,), (5, 1), (5, 1, 3), (5, 1, 3, 0)]:
    with DeviceTableau(0) as a, DeviceTableau(0) as b:
        a.set_window(K)
        a.load(T, basis)
        b.load(T, basis)
        for lim in lims:
            a.solve(max_iters=lim) if lim else a.solve()
        tb = b.tableau()
        bad = np.argwhere(tb != T)
        print(K, lims, "b corrupted cells:", len(bad), bad[:6].tolist(), flush=True)
