"""``linprog``-compatible adapter over the GPU tableau engine.

The reference gets its answer from
``scipy.optimize.linprog(c, A_ub=, b_ub=, A_eq=, b_eq=, bounds=,
method='highs-ds', options={'presolve': True, 'time_limit': 10})``
(app/controllers/solver_controller.py:76-85) and maps ``result.status`` at :404
(2 -> "Sin Solucion Factible", anything else unsuccessful -> "Error").  This
function accepts the same arguments and returns a ``scipy.optimize.OptimizeResult``
with the same fields (x, fun, success, status, message, nit), solved by the
two-phase tableau simplex of simplex_amd.lp on the GPU.  The controller can use
it in place of scipy's (``SolverController(..., answer_engine="gpu")``).

Bounds: each (lo, hi) pair with lo finite is shifted (x = lo + x'); hi < inf
adds the row x' <= hi - lo; lo = -inf (None) splits x = x+ - x-.  ``method``
and HiGHS-specific options are accepted and ignored, except ``time_limit`` and
``maxiter``.
"""
from __future__ import annotations

import math

import numpy as np
from scipy.optimize import OptimizeResult

from .lp import solve_lp

MESSAGES = {0: "Optimization terminated successfully. (GPU tableau simplex)",
            1: "Iteration or time limit reached. (GPU tableau simplex)",
            2: "The problem is infeasible. (GPU tableau simplex)",
            3: "The problem is unbounded. (GPU tableau simplex)"}


def _bounds_list(bounds, n):
    if bounds is None:
        return [(0.0, math.inf)] * n
    if isinstance(bounds, tuple) and len(bounds) == 2 and not isinstance(bounds[0], (list, tuple)):
        bounds = [bounds] * n
    out = []
    for b in bounds:
        lo, hi = (b if b is not None else (None, None))
        lo = -math.inf if lo is None else float(lo)
        hi = math.inf if hi is None else float(hi)
        if lo > hi:
            raise ValueError(f"infeasible bound {b}")
        out.append((lo, hi))
    if len(out) != n:
        raise ValueError(f"{len(out)} bounds for {n} variables")
    return out


def linprog(c, A_ub=None, b_ub=None, A_eq=None, b_eq=None, bounds=(0, None), method="highs-ds",
            callback=None, options=None, x0=None, integrality=None, *, device=0,
            rule="dantzig"):
    """Minimise c @ x subject to A_ub x <= b_ub, A_eq x == b_eq, bounds."""
    options = dict(options or {})
    c = np.asarray(c, dtype=np.float64).reshape(-1)
    n = c.shape[0]
    A_ub = np.zeros((0, n)) if A_ub is None else np.asarray(A_ub, dtype=np.float64).reshape(-1, n)
    b_ub = np.zeros(0) if b_ub is None else np.asarray(b_ub, dtype=np.float64).reshape(-1)
    A_eq = np.zeros((0, n)) if A_eq is None else np.asarray(A_eq, dtype=np.float64).reshape(-1, n)
    b_eq = np.zeros(0) if b_eq is None else np.asarray(b_eq, dtype=np.float64).reshape(-1)
    bl = _bounds_list(bounds, n)

    # variable map: x_j = shift_j + sum_k coef_jk * y_k  (y >= 0)
    cols, shift = [], np.zeros(n)
    extra_rows = []
    for j, (lo, hi) in enumerate(bl):
        if math.isfinite(lo):
            shift[j] = lo
            k = len(cols)
            cols.append((j, 1.0))
            if math.isfinite(hi):
                extra_rows.append((k, hi - lo))
        elif math.isfinite(hi):  # x = hi - y
            shift[j] = hi
            cols.append((j, -1.0))
        else:  # free: x = y+ - y-
            cols.append((j, 1.0))
            cols.append((j, -1.0))
    ny = len(cols)
    M = np.zeros((n, ny))
    for k, (j, s) in enumerate(cols):
        M[j, k] = s
    cy = c @ M
    rows = []
    for a, b in zip(A_ub, b_ub):
        rows.append((a @ M, "<=", b - a @ shift))
    for a, b in zip(A_eq, b_eq):
        rows.append((a @ M, "=", b - a @ shift))
    for k, ub in extra_rows:
        e = np.zeros(ny)
        e[k] = 1.0
        rows.append((e, "<=", ub))
    res = solve_lp(-cy, rows, maximize=True, device=device, rule=rule,
                   max_iters=int(options.get("maxiter", 0) or 0),
                   time_limit=float(options.get("time_limit", 0.0) or 0.0))
    out = OptimizeResult()
    out.status = int(res.status)
    out.success = res.status == 0
    out.message = MESSAGES.get(res.status, "error")
    out.nit = int(res.iters)
    if res.status == 0:
        x = shift + M @ res.x
        out.x = x
        out.fun = float(c @ x)
        slack = b_ub - A_ub @ x if A_ub.size else np.zeros(0)
        out.slack = slack
        out.con = b_eq - A_eq @ x if A_eq.size else np.zeros(0)
    else:
        out.x = None
        out.fun = None
    return out
