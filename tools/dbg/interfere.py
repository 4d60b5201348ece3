"""Does a lazy chain slow down while an HBM-bound elimination stream runs
beside it?  Context A: K=16 windows through the phase-probe library (lazy
kernel timestamps); context B (other stream, other host thread): back-to-back
single-pivot eliminations of a second config-3 tableau (~6.6 TB/s)."""
import ctypes, os, sys, threading, time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["SPX_LIB"] = os.path.join(ROOT, "simplex-solver_amd", "simplex_amd", "lib", "libspx_probe.so")
sys.path.insert(0, os.path.join(ROOT, "simplex-solver_amd"))
import numpy as np
from simplex_amd import synth
from simplex_amd.engine import DeviceTableau

m = n = 8192
Tf, obj, basis = synth.tableau_rows("dense", m, n, 20251205, order="F")
A = DeviceTableau(0); A.set_window(16); A.load_rows(Tf, obj, basis, m, 0)
B = DeviceTableau(0); B.load_rows(Tf, obj, basis, m, 0)
del Tf
lib = ctypes.CDLL(os.environ["SPX_LIB"])
NB = 1024 + 2 * 8192
buf = (ctypes.c_ulonglong * NB)()

def window_profile():
    A.run_pivots(16); A.sync()
    assert lib.spx_probe_read(buf, NB) == 0
    t = lambda slot, kind, ph: buf[((slot * 4 + kind) * 4 + ph) & 1023]
    t0 = t(0, 0, 0)
    lazy_end = (t(15, 1, 3) - t0) / 100.0
    kern = [(t(q, k, 3) - t(q, k, 0)) / 100.0 for q in range(16) for k in (0, 1)]
    f0 = (t(16, 2, 0) - t0) / 100.0
    f1 = (t(16, 2, 1) - t0) / 100.0
    return lazy_end, float(np.mean(kern)), f1 - f0

A.run_pivots(64); A.sync()
B.run_pivots(64); B.sync()
for label in ("alone", "beside elim stream", "alone"):
    stop = False
    def hog():
        while not stop:
            B.run_pivots(32); B.sync()
    th = None
    if label != "alone":
        th = threading.Thread(target=hog); th.start(); time.sleep(0.5)
    res = [window_profile() for _ in range(8)]
    stop = True
    if th: th.join()
    r = np.array(res)
    print(f"{label:20s} lazy chain {r[:,0].mean():7.1f} us  mean lazy kernel {r[:,1].mean():5.2f} us"
          f"  flush block0 {r[:,2].mean():6.1f} us", flush=True)
A.close(); B.close()
