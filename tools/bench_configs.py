"""Timings of the BASELINE.json configs other than the headline (bench.py is
config 3 / 4).  One JSON line per config:

  config 2: 1024 x 2048 dense random-feasible LP, full Dantzig solve on one GPU
            (wall time of spx_solve, hipGraph chunks), vs the C/OpenMP oracle's
            full solve and HiGHS (linprog 'highs-ds', the reference's answer
            path, solver_controller.py:78-85) on the host.
  config 5: degenerate 4096 x 4096 LP, Bland's rule: pivots/s over K pivots on
            one GPU vs the C/OpenMP oracle over its first pivots (same
            sequence checked).
  full solves (--full): config 3's Dantzig solve to optimality (22,169
            pivots) and config 5's 100,000-pivot Bland prefix on one GPU at
            K = 24, wall time of spx_solve with the tableau resident, beside
            the pinned fixture's oracle and HiGHS 'highs-ds' wall times
            (tests/golden/fullsize.json: measured in the dev container, 4
            oracle threads; HiGHS takes minutes there, so it is not re-run
            on the GPU box).  The GPU's pivot count and objective must equal
            the fixture's bit for bit.
All GPU results are checked against the oracle (objective / pivot sequence).
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "simplex-solver_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

from oracle import c_oracle as C  # noqa: E402
from simplex_amd import synth  # noqa: E402
from simplex_amd.engine import DeviceTableau as _DeviceTableau  # noqa: E402

PAD = int(os.environ.get("SPX_LD_PAD", "-1"))  # column padding override (A/B runs)


def DeviceTableau(dev):
    e = _DeviceTableau(dev)
    if PAD >= 0:
        e.set_ld_pad(PAD)
    return e


def config2(window=0):
    m, n, seed = 1024, 2048, 20251207
    T, basis = synth.full_tableau("dense", m, n, seed)
    with DeviceTableau(0) as e:
        e.set_window(window)
        e.load(T, basis)
        e.solve(max_iters=5)  # warm: graph build, first launches
        e.load(T, basis)
        t0 = time.perf_counter()
        res = e.solve()
        gpu_s = time.perf_counter() - t0
        hist = e.history().tolist()
    Tc, bc = T.copy(), basis.copy()
    t0 = time.perf_counter()
    st, hc = C.solve(Tc, bc)
    cpu_s = time.perf_counter() - t0
    from scipy.optimize import linprog
    A, b, c = synth.lp_data("dense", m, n, seed)
    t0 = time.perf_counter()
    h = linprog(-c, A_ub=A, b_ub=b, bounds=[(0, None)] * n, method="highs-ds")
    highs_s = time.perf_counter() - t0
    return {"config": "2: 1024x2048 dense LP, full Dantzig solve", "window": window,
            "gpu_s": gpu_s,
            "pivots": res.iters, "gpu_pivots_per_s": res.iters / gpu_s,
            "objective": res.objective, "highs_objective": -h.fun, "highs_s": highs_s,
            "highs_nit": int(h.nit), "cpu_oracle_s": cpu_s, "cpu_threads": C.threads(),
            "sequence_matches_oracle": [tuple(x) for x in hist] == hc,
            "objective_rel_err_vs_highs": abs(res.objective + h.fun) / abs(h.fun)}


def config5(window=0, k=2048, k_cpu=60):
    m = n = 4096
    T, basis = synth.full_tableau("degenerate", m, n, 5)
    with DeviceTableau(0) as e:
        e.set_window(window)
        e.load(T, basis)
        e.run_pivots(20, rule="bland")
        e.sync()
        t0 = time.perf_counter()
        e.run_pivots(k, rule="bland")
        e.sync()
        gpu_s = time.perf_counter() - t0
        st, it, z = e.state()
        hist = e.history().tolist()
    Tc, bc = T.copy(), basis.copy()
    t0 = time.perf_counter()
    stc, hc = C.solve(Tc, bc, rule="bland", max_iters=k_cpu)
    cpu_s = time.perf_counter() - t0
    return {"config": "5: degenerate 4096x4096 LP, Bland", "window": window, "gpu_pivots": k,
            "ld_pad": PAD,
            "gpu_pivots_per_s": k / gpu_s, "status_after": st, "iters": it,
            "cpu_oracle_pivots_per_s": len(hc) / cpu_s, "cpu_threads": C.threads(),
            "first_pivots_match_oracle": [tuple(x) for x in hist[:len(hc)]] == hc}


def full_solve(name, window=24):
    fx = json.load(open(os.path.join(ROOT, "tests", "golden", "fullsize.json")))[name]
    cap = fx.get("max_pivots", 0)
    Tf, obj, basis = synth.tableau_rows(fx["kind"], fx["m"], fx["n"], fx["seed"], order="F")
    with DeviceTableau(0) as e:
        e.set_window(window)
        e.load_rows(Tf, obj, basis, fx["m"], 0)
        e.solve(rule=fx["rule"], max_iters=2 * window)  # warm: graphs, first launches
        e.load_rows(Tf, obj, basis, fx["m"], 0)
        del Tf
        t0 = time.perf_counter()
        res = e.solve(rule=fx["rule"], max_iters=cap)
        gpu_s = time.perf_counter() - t0
    return {"config": f"{name}: {fx['m']}x{fx['n']} {fx['kind']} LP, {fx['rule']}, "
                      + (f"first {cap} pivots" if cap else "solve to optimality"),
            "window": window, "ld_pad": PAD, "gpu_s": gpu_s, "pivots": res.iters,
            "gpu_pivots_per_s": res.iters / gpu_s, "status": res.status,
            "objective": res.objective, "matches_fixture": res.iters == fx["pivots"]
            and res.objective == fx["objective"],
            "oracle_s_dev_container": fx.get("oracle_seconds"),
            "oracle_threads_dev_container": fx.get("oracle_threads"),
            "highs_s_dev_container": fx.get("highs_seconds"), "highs_nit": fx.get("highs_nit"),
            "highs_objective": fx.get("highs_objective"),
            "highs_note": "HiGHS solves the LP to optimality (a different algorithm)"
                          + ("; the GPU runs the fixture's Bland prefix" if cap else "")}


if __name__ == "__main__":
    if "--config5-k24" in sys.argv:
        print(json.dumps(config5(24, k=8192)), flush=True)
        sys.exit(0)
    if "--full" in sys.argv:
        for name in ("config3", "config5"):
            print(json.dumps(full_solve(name)), flush=True)
        sys.exit(0)
    for fn, w in ((config2, 0), (config2, 8), (config2, 24), (config5, 0), (config5, 16), (config5, 24)):
        print(json.dumps(fn(w)), flush=True)
