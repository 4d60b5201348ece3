"""CPU oracle of the dense tableau simplex — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module, and only as the checker / the timed CPU baseline.  The product
path (simplex-solver_amd/simplex_amd) never imports it.

What it restates
  The reference's tableau pivot loop lives in the third-party package
  ``simple_simplex==0.0.3`` (reference requirements.txt:10), imported at
  app/controllers/solver_controller.py:22-27, driven at :290-319 and whose
  ``pivotSteps`` are consumed at :322-363.  That package is not vendored under
  /root/reference and cannot be installed offline, so its exact arithmetic is
  unreadable.  This oracle restates the build's written spec,
  which follows the north star's description of that loop: entering column by
  most-negative reduced cost (Dantzig) or Bland's rule, min-ratio leaving row,
  Gauss-Jordan elimination over the full (m+1) x (n+m+1) tableau.

Pinning ("parity" status)
  * Pivot sequence / tableau / basis: PARITY UNPINNED against simple_simplex
    (unavailable, no reference test asserts on pivotSteps).
  * Objective / status / x: pinned against the reference tests' known answers
    that are true optima (tests/test_solver_controller.py:32-46,
    tests/test_visualization_integration.py:38-56, :208-224, :243-259,
    :349-362, :379-395, tests/test_ui_controller.py:28-41) and against HiGHS
    (scipy.optimize.linprog(method='highs-ds'), the reference's answer path at
    solver_controller.py:76-85) on generated LPs.  See tests/golden/.

Spec (bit-exact conventions)
  tableau T: (m+1) x N, objective row last ("z_j - c_j" of a MAX problem),
  RHS in column N-1.
  enter  : Dantzig -> argmin over j < n_enter with T[m,j] < -eps_opt of
           (T[m,j], j); Bland -> smallest such j.  None -> optimal.
  leave  : rows i with T[i,c] > eps_piv, ratio T[i,N-1] / T[i,c] (IEEE
           division, NaN ratios ignored); Dantzig -> min (ratio, i); Bland ->
           min (ratio, basis[i]).  None -> unbounded.
  pivot  : p = T[r,:] / T[r,c]; f = T[:,c] (copy); for every column j with
           p[j] != 0 (all columns when skip_zero=False) and every row i != r:
           T[i,j] = T[i,j] - (f[i] * p[j])  (rounded product, then rounded
           difference: no FMA); T[r,j] = p[j]; then column c = e_r.  Columns
           with p[j] == 0 are left untouched (identical to the dense update up
           to the sign of zero).
"""
from __future__ import annotations

import numpy as np

OPTIMAL, ITER_LIMIT, INFEASIBLE, UNBOUNDED = 0, 1, 2, 3
DANTZIG, BLAND = "dantzig", "bland"
DRIVE_OUT_TOL = 1e-9


# --------------------------------------------------------------------- steps
def select_entering(obj_row: np.ndarray, n_enter: int, rule: str, eps_opt: float):
    z = obj_row[:n_enter]
    cand = np.flatnonzero(z < -eps_opt)
    if cand.size == 0:
        return None
    if rule == BLAND:
        return int(cand[0])
    return int(cand[np.argmin(z[cand])])  # first occurrence = lowest column on ties


def ratio_test(T: np.ndarray, c: int, basis: np.ndarray, rule: str, eps_piv: float):
    m = T.shape[0] - 1
    if m == 0:
        return None
    col = T[:m, c]
    rows = np.flatnonzero(col > eps_piv)
    if rows.size == 0:
        return None
    ratios = T[rows, -1] / col[rows]
    keep = ~np.isnan(ratios)
    rows, ratios = rows[keep], ratios[keep]
    if rows.size == 0:
        return None
    if rule == BLAND:
        tied = rows[ratios == ratios.min()]
        return int(tied[np.argmin(basis[tied])])
    return int(rows[np.argmin(ratios)])  # first occurrence = lowest row


def pivot(T: np.ndarray, r: int, c: int, skip_zero: bool = True, block_rows: int = 256) -> int:
    """In-place Gauss-Jordan pivot on (r, c).  Returns the number of columns
    updated (the elimination's touched columns)."""
    piv = T[r, c]
    p = T[r, :] / piv
    f = T[:, c].copy()
    cols = np.flatnonzero(p != 0.0) if skip_zero else np.arange(T.shape[1])
    pn = p[cols]
    rows = T.shape[0]
    for i0 in range(0, rows, block_rows):
        i1 = min(rows, i0 + block_rows)
        blk = T[i0:i1][:, cols]
        blk -= np.multiply.outer(f[i0:i1], pn)
        T[i0:i1, cols] = blk
    T[r, cols] = pn
    T[:, c] = 0.0
    T[r, c] = 1.0
    return int(cols.size)


def solve_tableau(T: np.ndarray, basis: np.ndarray, rule: str = DANTZIG, eps_opt: float = 1e-9,
                  eps_piv: float = 1e-12, n_enter: int | None = None, max_iters: int = 0,
                  skip_zero: bool = True, on_pivot=None):
    """Phase loop on T (in place).  Returns (status, history[(r, c)])."""
    n_enter = T.shape[1] - 1 if n_enter is None else n_enter
    hist = []
    while True:
        if max_iters and len(hist) >= max_iters:
            return ITER_LIMIT, hist
        c = select_entering(T[-1], n_enter, rule, eps_opt)
        if c is None:
            return OPTIMAL, hist
        r = ratio_test(T, c, basis, rule, eps_piv)
        if r is None:
            return UNBOUNDED, hist
        pivot(T, r, c, skip_zero)
        basis[r] = c
        hist.append((r, c))
        if on_pivot is not None:
            on_pivot(r, c, T)


# --------------------------------------------------------------- standard form
def standard_form(c, rows, maximize: bool):
    """Restatement of the build's standard form.
    Returns dict(T, basis, n, m, k, cost, art_rows)."""
    flip = {"L": "G", "G": "L", "E": "E"}
    opmap = {"<=": "L", ">=": "G", "=": "E", "L": "L", "G": "G", "E": "E"}
    c = np.asarray(c, dtype=np.float64).reshape(-1)
    n, m = c.shape[0], len(rows)
    A = np.zeros((m, n))
    b = np.zeros(m)
    ops = []
    for i, (a, op, rhs) in enumerate(rows):
        a = np.asarray(a, dtype=np.float64).reshape(-1)
        o = opmap[op]
        rhs = float(rhs)
        if rhs < 0:
            a, rhs, o = -a, -rhs, flip[o]
        A[i], b[i] = a, rhs
        ops.append(o)
    art = [i for i, o in enumerate(ops) if o != "L"]
    k = len(art)
    N = n + m + k + 1
    T = np.zeros((m + 1, N))
    T[:m, :n] = A
    T[:m, -1] = b
    basis = np.zeros(m, dtype=np.int64)
    for i, o in enumerate(ops):
        if o == "L":
            T[i, n + i] = 1.0
            basis[i] = n + i
        elif o == "G":
            T[i, n + i] = -1.0
    for q, i in enumerate(art):
        T[i, n + m + q] = 1.0
        basis[i] = n + m + q
    cost = np.zeros(N - 1)
    cost[:n] = c if maximize else -c
    if k == 0:
        T[m, :N - 1] = -cost
    else:
        w = np.zeros(N)
        w[n + m:n + m + k] = 1.0
        for i in art:
            w = w - T[i]
        T[m] = w
    return dict(T=T, basis=basis, n=n, m=m, k=k, cost=cost, art_rows=art, maximize=maximize)


def phase2_row(T, basis, cost):
    N = T.shape[1]
    obj = np.zeros(N)
    obj[:N - 1] = -cost
    for i in range(T.shape[0] - 1):
        cb = cost[basis[i]]
        if cb != 0.0:
            obj = obj + cb * T[i]
    return obj


def solve_lp(c, rows, maximize=True, rule=DANTZIG, max_iters=0):
    """Two-phase restatement.  Returns dict(status, x, objective, pivots, T, basis)."""
    sf = standard_form(c, rows, maximize)
    T, basis, n, m, k = sf["T"], sf["basis"], sf["n"], sf["m"], sf["k"]
    n_enter = n + m
    pivots = []
    if k:
        st, h = solve_tableau(T, basis, rule, n_enter=n_enter, max_iters=max_iters)
        pivots += [(1, r, c_) for r, c_ in h]
        if st == ITER_LIMIT:
            return dict(status=ITER_LIMIT, x=None, objective=None, pivots=pivots, T=T,
                        basis=basis)
        bmax = float(np.max(np.abs(sf["T"][:m, -1]))) if m else 0.0
        if T[-1, -1] < -1e-9 * (1.0 + bmax):
            return dict(status=INFEASIBLE, x=None, objective=None, pivots=pivots, T=T,
                        basis=basis)
        for i in range(m):
            if basis[i] >= n_enter:
                cand = np.flatnonzero(np.abs(T[i, :n_enter]) > DRIVE_OUT_TOL)
                if cand.size:
                    j = int(cand[0])
                    pivot(T, i, j)
                    basis[i] = j
                    pivots.append((1, i, j))
        T[-1] = phase2_row(T, basis, sf["cost"])
    st, h = solve_tableau(T, basis, rule, n_enter=n_enter,
                          max_iters=(max_iters - len(pivots)) if max_iters else 0)
    pivots += [(2, r, c_) for r, c_ in h]
    if st != OPTIMAL:
        return dict(status=st, x=None, objective=None, pivots=pivots, T=T, basis=basis)
    x = np.zeros(n)
    for i, j in enumerate(basis):
        if j < n:
            x[j] = T[i, -1]
    z = T[-1, -1] if maximize else -T[-1, -1]
    return dict(status=OPTIMAL, x=x, objective=float(z), pivots=pivots, T=T, basis=basis)
