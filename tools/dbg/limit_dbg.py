import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "simplex-solver_amd")); sys.path.insert(0, ROOT)
import numpy as np
from simplex_amd import synth
from simplex_amd.engine import DeviceTableau
from oracle import simplex_oracle as O
T, basis = synth.full_tableau("dense", 64, 96, 7)
ref, rb = T.copy(), basis.copy()
st, hist = O.solve_tableau(ref, rb, max_iters=12)
print("oracle", hist[:12])
for lims in [(12,), (5,), (4,), (5, 1, 3), (2, 2)]:
    with DeviceTableau(0) as a:
        a.set_window(4)
        a.load(T, basis)
        out = []
        for lim in lims:
            r = a.solve(max_iters=lim)
            out.append((r.status, r.iters))
        print(lims, out, [tuple(x) for x in a.history().tolist()])
with DeviceTableau(0) as b:
    b.load(T, basis)
    b.solve(max_iters=12)
    print("plain", [tuple(x) for x in b.history().tolist()])
