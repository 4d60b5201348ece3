"""Windowed-flush variant sweep on the config-3 tableau, one process.

For each window size K and flush variant (rows/thread x columns/step, see
spx_capi.hip), runs S pivots with HIP events around every flush and prints the
average flush time, the touched columns per flush and the end-to-end pivots/s.
Rounds are interleaved so drift in the LP state affects every variant alike.

usage: python tools/tune_flush.py [--ks 16,32] [--fvs 0,1,2,3,4] [--steps 128] [--rounds 2]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "simplex-solver_amd"))
if "--probe-lib" in sys.argv:  # the phase-timing build of tools/probe_phases.py
    os.environ["SPX_LIB"] = os.path.join(ROOT, "simplex-solver_amd", "simplex_amd", "lib",
                                         "libspx_probe.so")
# (every variant 0-7 is dispatched by the main libspx.so; 1-5 only for
# power-of-two K, other K fall back to the default LDS-DMA ring)

from simplex_amd import synth  # noqa: E402
from simplex_amd.engine import DeviceTableau  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ks", default="16,32")
    ap.add_argument("--fvs", default="0,1,2,3,4")
    ap.add_argument("--steps", type=int, default=128)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--m", type=int, default=8192)
    ap.add_argument("--n", type=int, default=8192)
    ap.add_argument("--wgs", type=int, default=0)
    ap.add_argument("--probe-lib", action="store_true")
    a = ap.parse_args()
    Tf, obj, basis = synth.tableau_rows("dense", a.m, a.n, 20251205, order="F")
    e = DeviceTableau(0)
    e.load_rows(Tf, obj, basis, a.m, 0)
    del Tf
    e.run_pivots(16)
    e.sync()
    for rnd in range(a.rounds):
        for K in [int(x) for x in a.ks.split(",")]:
            for fv in [int(x) for x in a.fvs.split(",")]:
                e.set_window(K)
                e.set_elim_variant(0, a.wgs, -1, flush_variant=fv & 7, flush_map=fv >> 3)
                e.run_pivots(2 * K)
                e.sync()
                e.elim_timing(reset=True)
                t0 = time.perf_counter()
                e.run_pivots(a.steps, time_elim=1)
                e.sync()
                el = time.perf_counter() - t0
                ms, cnt, cols = e.elim_timing(reset=True)
                st, it, _ = e.state()
                print(json.dumps({"round": rnd, "K": K, "fv": fv, "flush_us": 1e3 * ms / cnt,
                                  "cols_per_flush": cols / cnt, "pivots_per_s": a.steps / el,
                                  "status": st, "iters": it}), flush=True)
    e.close()


if __name__ == "__main__":
    main()
