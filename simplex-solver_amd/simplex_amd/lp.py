"""LP model -> simplex tableau, and the two-phase driver over DeviceTableau.

The reference hands an LP to its pivot engine as text rows
(app/controllers/solver_controller.py:302-316: ``"a1,..,an,{L|G|E},b"`` per
constraint, ``"c1,..,cn,{1|0}"`` for the objective) and expects the optimum
plus a per-pivot tableau history back (``optimize_json_format``, :318,
consumed at :322-363).  This module fixes the tableau those rows become
("standard form") and drives the GPU engine through phase 1
(artificial variables, for ``>=`` / ``=`` rows and negative right-hand sides)
and phase 2.

Standard form
  * a row with b < 0 is multiplied by -1 (L <-> G swap, E stays);
  * columns: x_0..x_{n-1} | s_0..s_{m-1} | a_0..a_{k-1} | RHS, where s_i is
    +1 (L row), -1 (G row) or an all-zero column (E row), and one artificial
    a is appended per G/E row in row order;
  * initial basis: s_i for L rows, the row's artificial otherwise;
  * MAX form: cost = c (maximize) or -c (minimize); objective row = -cost
    (z_j - c_j), RHS = objective value.
Phase 1 maximises -sum(a) from the canonical row e_art - sum(artificial rows);
artificials never re-enter (n_enter = n + m).  Basic artificials left at zero
are driven out by a pivot on the first non-artificial column with |T[i,j]| >
1e-9.  Phase 2's row is -cost + sum_i cost[basis[i]] * T[i,:] accumulated
row by row in order (elementwise, no BLAS, so every implementation rounds it
identically).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Callable, List, Optional, Sequence

import numpy as np

from .engine import POOL, DeviceTableau, SolveResult, auto_window
from . import _lib as L

OPS = {"<=": "L", "L": "L", ">=": "G", "G": "G", "=": "E", "==": "E", "E": "E"}
FLIP = {"L": "G", "G": "L", "E": "E"}
DRIVE_OUT_TOL = 1e-9


@dataclass
class StandardForm:
    T: np.ndarray            # (m+1) x N initial tableau, objective row last
    basis: np.ndarray        # m int64
    n: int                   # structural variables
    m: int                   # constraints
    k: int                   # artificial variables
    cost: np.ndarray         # N-1 MAX-form costs (0 off the structural block)
    maximize: bool
    art_rows: List[int]
    phase2_obj: Optional[np.ndarray] = None  # set when k == 0

    @property
    def N(self) -> int:
        return self.T.shape[1]

    @property
    def n_enter(self) -> int:
        return self.n + self.m


def build_standard_form(c: Sequence[float], rows: Sequence[tuple], maximize: bool) -> StandardForm:
    """rows = [(coeffs (n,), op in {'<=','>=','=','L','G','E'}, rhs), ...]."""
    c = np.asarray(c, dtype=np.float64).reshape(-1)
    n = c.shape[0]
    m = len(rows)
    A = np.zeros((m, n), dtype=np.float64)
    b = np.zeros(m, dtype=np.float64)
    ops = []
    for i, (a, op, rhs) in enumerate(rows):
        a = np.asarray(a, dtype=np.float64).reshape(-1)
        if a.shape[0] != n:
            raise ValueError(f"constraint {i} has {a.shape[0]} coefficients, expected {n}")
        if op not in OPS:
            raise ValueError(f"constraint {i}: unknown operator {op!r}")
        o = OPS[op]
        rhs = float(rhs)
        if rhs < 0:
            a, rhs, o = -a, -rhs, FLIP[o]
        A[i] = a
        b[i] = rhs
        ops.append(o)
    art_rows = [i for i, o in enumerate(ops) if o in ("G", "E")]
    k = len(art_rows)
    N = n + m + k + 1
    T = np.zeros((m + 1, N), dtype=np.float64)
    T[:m, :n] = A
    T[:m, N - 1] = b
    basis = np.empty(m, dtype=np.int64)
    for i, o in enumerate(ops):
        if o == "L":
            T[i, n + i] = 1.0
            basis[i] = n + i
        elif o == "G":
            T[i, n + i] = -1.0
    for q, i in enumerate(art_rows):
        T[i, n + m + q] = 1.0
        basis[i] = n + m + q
    cost = np.zeros(N - 1, dtype=np.float64)
    cost[:n] = c if maximize else -c
    if k == 0:
        T[m, :N - 1] = -cost
        sf = StandardForm(T, basis, n, m, 0, cost, bool(maximize), art_rows)
        sf.phase2_obj = T[m].copy()
        return sf
    obj1 = np.zeros(N, dtype=np.float64)
    obj1[n + m:n + m + k] = 1.0
    for i in art_rows:
        obj1 = obj1 - T[i]
    T[m] = obj1
    return StandardForm(T, basis, n, m, k, cost, bool(maximize), art_rows)


def phase2_objective(T: np.ndarray, basis: np.ndarray, cost: np.ndarray) -> np.ndarray:
    """-cost + sum_i cost[basis[i]] * T[i, :], accumulated in row order."""
    m = T.shape[0] - 1
    N = T.shape[1]
    obj = np.zeros(N, dtype=np.float64)
    obj[:N - 1] = -cost
    for i in range(m):
        cb = cost[basis[i]]
        if cb != 0.0:
            obj = obj + cb * T[i]
    return obj


@dataclass
class LPResult:
    status: int                      # 0 optimal, 1 limit, 2 infeasible, 3 unbounded
    x: Optional[np.ndarray]          # structural values (None unless optimal)
    objective: Optional[float]       # in the caller's sense (max or min)
    iters: int
    basis: Optional[np.ndarray] = None
    pivots: List[tuple] = field(default_factory=list)   # (phase, row, col)
    steps: List[dict] = field(default_factory=list)     # pivotSteps when recorded

    @property
    def success(self) -> bool:
        return self.status == 0


def _extract(sf: StandardForm, T_rhs: np.ndarray, basis: np.ndarray) -> np.ndarray:
    x = np.zeros(sf.n, dtype=np.float64)
    for i, j in enumerate(basis):
        if j < sf.n:
            x[j] = T_rhs[i]
    return x


class _Recorder:
    """Collects pivotSteps snapshots under a cell budget."""

    def __init__(self, eng: DeviceTableau, enabled: bool, cell_budget: int):
        self.eng = eng
        self.enabled = enabled
        self.budget = cell_budget
        self.steps: List[dict] = []
        self.step = 0

    def snapshot_ok(self) -> bool:
        cells = (self.eng.m_local + 1) * self.eng.N
        return self.enabled and self.budget >= cells

    def record(self, r, c, phase, force=False):
        if not self.enabled:
            return
        entry = {"step": self.step, "pivotRowIndex": r, "pivotColIndex": c, "phase": phase,
                 "tableau": []}
        if self.snapshot_ok() or force:
            entry["tableau"] = self.eng.tableau().tolist()
            self.budget -= (self.eng.m_local + 1) * self.eng.N
        self.steps.append(entry)
        self.step += 1


def _run_phase(eng: DeviceTableau, rec: _Recorder, phase: int, rule: str, n_enter: int,
               max_iters: int, time_limit: float, pivots: list, window: int = 0) -> SolveResult:
    """Pivot until optimal/unbounded/limit.  Snapshots one pivot at a time
    while the recorder's budget lasts, then hands the rest to spx_solve, in
    K-pivot windows when `window` > 1 (bit-identical)."""
    done = 0
    while rec.snapshot_ok() and (max_iters <= 0 or done < max_iters):
        out = eng.pivot(rule=rule, n_enter=n_enter)
        if not isinstance(out, tuple):
            st, _, z = eng.state()
            return SolveResult(out, done, z, 0.0)
        done += 1
        pivots.append((phase, out[0], out[1]))
        rec.record(out[0], out[1], phase)
    if max_iters > 0 and done >= max_iters:
        st, _, z = eng.state()
        return SolveResult(L.SPX_ITER_LIMIT, done, z, 0.0)
    before = eng.history().shape[0]
    if window > 1:
        eng.set_window(window)
    try:
        res = eng.solve(rule=rule, n_enter=n_enter,
                        max_iters=(max_iters - done) if max_iters > 0 else 0,
                        time_limit=time_limit)
    finally:
        if window > 1:
            eng.set_window(0)
    hist = eng.history()
    for r, c in hist[before:]:
        pivots.append((phase, int(r), int(c)))
    if rec.enabled and res.iters:
        # steps past the snapshot budget: indices only, final tableau kept
        for r, c in hist[before:]:
            rec.steps.append({"step": rec.step, "pivotRowIndex": int(r),
                              "pivotColIndex": int(c), "phase": phase, "tableau": []})
            rec.step += 1
    res.iters += done
    return res


def solve_standard_form(sf: StandardForm, *, device: int = 0, rule: str = "dantzig",
                        max_iters: int = 0, time_limit: float = 0.0, record: bool = False,
                        cell_budget: int = 2_000_000, window: int = -1,
                        engine_factory: Optional[Callable[[], DeviceTableau]] = None) -> LPResult:
    """Two-phase tableau simplex of a StandardForm on the GPU engine.
    window: pivots per tableau pass for the unrecorded stretch of each phase
    (-1: auto_window by size; 0: one pass per pivot)."""
    # (a pooled context unless the caller brings its own: engine.ContextPool)
    eng = engine_factory() if engine_factory else POOL.acquire(device)
    reusable = True  # (a context whose solve raised is destroyed, never pooled)
    if window < 0:
        window = auto_window(sf.m, sf.N)
    try:
        eng.load(sf.T, sf.basis)
        rec = _Recorder(eng, record, cell_budget)
        rec.record(None, None, 1 if sf.k else 2)
        pivots: list = []
        iters = 0
        if sf.k:
            res = _run_phase(eng, rec, 1, rule, sf.n_enter, max_iters, time_limit, pivots,
                             window)
            iters += res.iters
            if res.status == L.SPX_ITER_LIMIT:
                return LPResult(L.SPX_ITER_LIMIT, None, None, iters, eng.basis(), pivots,
                                rec.steps)
            bmax = float(np.max(np.abs(sf.T[:sf.m, -1]))) if sf.m else 0.0
            if eng.objective_row()[-1] < -1e-9 * (1.0 + bmax):
                return LPResult(L.SPX_INFEASIBLE, None, None, iters, eng.basis(), pivots,
                                rec.steps)
            # drive basic artificials (at zero level) out, one device row at a time
            basis = eng.basis()
            for i in range(sf.m):
                if basis[i] >= sf.n_enter:
                    cand = np.flatnonzero(np.abs(eng.row(i)[:sf.n_enter]) > DRIVE_OUT_TOL)
                    if cand.size:
                        j = int(cand[0])
                        eng.pivot_at(i, j)
                        iters += 1
                        pivots.append((1, i, j))
                        rec.record(i, j, 1)
                        basis = eng.basis()
            eng.set_phase2_objective(sf.cost)  # == phase2_objective(T, basis, cost)
            rec.record(None, None, 2)
        res = _run_phase(eng, rec, 2, rule, sf.n_enter,
                         (max_iters - iters) if max_iters > 0 else 0, time_limit, pivots,
                         window)
        iters += res.iters
        if rec.enabled and rec.steps and not rec.steps[-1]["tableau"]:
            rec.steps[-1]["tableau"] = eng.tableau().tolist()
        basis = eng.basis()
        if res.status != L.SPX_OPTIMAL:
            return LPResult(res.status, None, None, iters, basis, pivots, rec.steps)
        rhs = eng.column(sf.N - 1) if sf.m else np.zeros(0)
        x = _extract(sf, rhs, basis)
        zmax = eng.objective_row()[-1]
        z = float(zmax if sf.maximize else -zmax)
        return LPResult(L.SPX_OPTIMAL, x, z, iters, basis, pivots, rec.steps)
    except BaseException:
        reusable = False
        raise
    finally:
        if engine_factory:
            eng.close()
        else:
            POOL.release(eng, reusable)


def solve_lp(c, rows, maximize=True, **kw) -> LPResult:
    return solve_standard_form(build_standard_form(c, rows, maximize), **kw)
