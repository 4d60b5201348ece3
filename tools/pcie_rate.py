"""PCIe-inclusive rates of the boundary (diagnostic; not part of the product).

The C-ABI takes host buffers (spx_load / spx_load_rows copy the tableau to
HBM; spx_get_* copy results back), while bench.py's `value` is timed with the
tableau resident in HBM.  This tool times, on the config-3 tableau
(8192 x 16385 fp64, 1.07 GB), the host -> HBM load, the bench's workload (K = 24
windows), a whole solve to optimality, and the reads a caller makes after a
solve (objective row + basis, or the whole tableau), and prints one JSON line
with the PCIe-inclusive pivots/s beside the resident ones.

usage: python tools/pcie_rate.py [--windows 20] [--full]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "simplex-solver_amd"))

import numpy as np  # noqa: E402

from simplex_amd import synth  # noqa: E402
from simplex_amd.engine import DeviceTableau  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--windows", type=int, default=20)
    ap.add_argument("--full", action="store_true", help="also solve to optimality")
    ap.add_argument("--order", default="F", choices=["F", "C"],
                    help="host layout of the tableau: F column-major, C row-major (numpy's default)")
    a = ap.parse_args()
    K, m, n, seed = 24, 8192, 8192, 20251205
    Tf, obj, basis = synth.tableau_rows("dense", m, n, seed, order=a.order)
    nbytes = Tf.nbytes + obj.nbytes
    out = {"tool": "pcie_rate", "config": "config 3: 8192x16385 fp64", "window": K,
           "host_order": a.order,
           "tableau_bytes": int(nbytes)}
    with DeviceTableau(0) as e:
        e.set_window(K)
        e.load_rows(Tf, obj, basis, m, 0)  # warm: allocation, graphs
        e.run_pivots(2 * K)
        e.sync()
        t0 = time.perf_counter()
        e.load_rows(Tf, obj, basis, m, 0)
        e.sync()
        t_load = time.perf_counter() - t0
        t0 = time.perf_counter()
        e.run_pivots(a.windows * K)
        e.sync()
        t_run = time.perf_counter() - t0
        t0 = time.perf_counter()
        z = e.objective_row()
        b = e.basis()
        t_small = time.perf_counter() - t0
        t0 = time.perf_counter()
        T = e.tableau()
        t_tab = time.perf_counter() - t0
        piv = a.windows * K
        out.update({
            "load_s": t_load, "load_GBps": nbytes / t_load / 1e9,
            "readback_tableau_s": t_tab, "readback_GBps": T.nbytes / t_tab / 1e9,
            "readback_objective_basis_s": t_small,
            "bench_pivots": piv, "bench_resident_s": t_run,
            "bench_resident_pivots_per_s": piv / t_run,
            "bench_pcie_inclusive_pivots_per_s": piv / (t_load + t_run + t_small),
            "bench_pcie_inclusive_with_tableau_pivots_per_s": piv / (t_load + t_run + t_tab),
        })
        del T, z, b
        if a.full:
            e.load_rows(Tf, obj, basis, m, 0)
            e.sync()
            t0 = time.perf_counter()
            r = e.solve(use_graph=True)
            t_solve = time.perf_counter() - t0
            t0 = time.perf_counter()
            e.objective_row()
            e.basis()
            t_small2 = time.perf_counter() - t0
            out.update({"solve_pivots": int(r.iters), "solve_status": int(r.status),
                        "solve_resident_s": t_solve,
                        "solve_resident_pivots_per_s": r.iters / t_solve,
                        "solve_pcie_inclusive_pivots_per_s":
                            r.iters / (t_load + t_solve + t_small2)})
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
