"""Drop-in for the four ``simple_simplex`` (0.0.3) names the reference imports.

Reference call sites (app/controllers/solver_controller.py):
  :22-27   from simple_simplex import create_tableau, add_constraint,
           add_objective, optimize_json_format
  :297-300 create_tableau(number_of_variables=n, number_of_constraints=m)
  :302-309 add_constraint(tableau, "a1,...,an,{L|G|E},b")   (one per row)
  :311-316 add_objective(tableau, "c1,...,cn,{1|0}")        (1 = maximize)
  :318     optimize_json_format(tableau, maximize=bool)
  :322-363 consumes result["pivotSteps"][k] keys "step", "pivotRowIndex",
           "pivotColIndex", "tableau" (list of rows, objective row last).

``simple_simplex`` itself is not vendored and not installable offline, so the
pivot semantics here are this build's documented spec, executed
by the GPU engine (libspx.so via simplex_amd.engine) — there is no CPU path.
Errors are raised as Python exceptions, as the reference's Plan B expects
(solver_controller.py:203-205 catches them).
"""
from __future__ import annotations

from typing import List, Optional

from .lp import build_standard_form, solve_standard_form

STATUS_TEXT = {0: "optimal", 1: "iteration_limit", 2: "infeasible", 3: "unbounded"}

#: total tableau cells kept as pivotSteps snapshots per solve (a 8192x16384
#: tableau is 1 GB; the reference consumer renders every cell, :341-355)
HISTORY_CELL_BUDGET = 2_000_000


class SimplexTableau:
    """Mutable problem builder returned by create_tableau (in-place API)."""

    def __init__(self, number_of_variables: int, number_of_constraints: int):
        if number_of_variables < 0 or number_of_constraints < 0:
            raise ValueError("sizes must be non-negative")
        self.n = int(number_of_variables)
        self.m = int(number_of_constraints)
        self.rows: List[tuple] = []
        self.c: Optional[list] = None
        self.maximize_flag: Optional[bool] = None

    def __repr__(self):
        return (f"SimplexTableau(n={self.n}, m={self.m}, rows={len(self.rows)}, "
                f"objective={'set' if self.c is not None else 'unset'})")


def _floats(tokens, what):
    try:
        return [float(t) for t in tokens]
    except ValueError as e:
        raise ValueError(f"{what}: non-numeric coefficient ({e})") from None


def create_tableau(number_of_variables: int, number_of_constraints: int) -> SimplexTableau:
    return SimplexTableau(number_of_variables, number_of_constraints)


def add_constraint(tableau: SimplexTableau, constraint: str) -> None:
    """``"a1,...,an,{L|G|E},b"`` (the string built at solver_controller.py:303-308)."""
    toks = [t.strip() for t in str(constraint).split(",")]
    if len(toks) != tableau.n + 2:
        raise ValueError(f"constraint {constraint!r}: expected {tableau.n} coefficients, "
                         "an operator and a right-hand side")
    op = toks[tableau.n].upper()
    if op not in ("L", "G", "E"):
        raise ValueError(f"constraint {constraint!r}: operator must be L, G or E")
    if len(tableau.rows) >= tableau.m:
        raise ValueError(f"tableau was created for {tableau.m} constraints")
    coeffs = _floats(toks[:tableau.n], "constraint")
    rhs = _floats([toks[tableau.n + 1]], "constraint")[0]
    tableau.rows.append((coeffs, op, rhs))


def add_objective(tableau: SimplexTableau, objective: str) -> None:
    """``"c1,...,cn,{1|0}"`` (solver_controller.py:311-315): the trailing token
    is the sense flag the controller writes (1 = maximize)."""
    toks = [t.strip() for t in str(objective).split(",")]
    if len(toks) != tableau.n + 1:
        raise ValueError(f"objective {objective!r}: expected {tableau.n} coefficients "
                         "and a sense flag")
    tableau.c = _floats(toks[:tableau.n], "objective")
    flag = toks[tableau.n]
    if flag not in ("0", "1", "0.0", "1.0"):
        raise ValueError(f"objective {objective!r}: sense flag must be 1 (max) or 0 (min)")
    tableau.maximize_flag = float(flag) == 1.0


def optimize_json_format(tableau: SimplexTableau, maximize: Optional[bool] = None,
                         rule: str = "dantzig", device: int = 0, max_iters: int = 0,
                         time_limit: float = 0.0) -> dict:
    """Solve on the GPU engine and return ``{"pivotSteps": [...], ...}``.

    pivotSteps[0] is the initial tableau (pivot indices None); step k >= 1 is
    the tableau AFTER the k-th pivot (pivotRowIndex, pivotColIndex), 0-based.
    Two-phase problems add a step with pivot None where phase 2 starts.
    Snapshots stop after HISTORY_CELL_BUDGET cells (later steps carry only the
    indices and an empty "tableau"; the final tableau is always present).
    """
    if tableau.c is None:
        raise ValueError("add_objective must be called before optimize_json_format")
    if len(tableau.rows) != tableau.m:
        raise ValueError(f"{len(tableau.rows)} of {tableau.m} constraints were added")
    if maximize is None:
        maximize = bool(tableau.maximize_flag)
    sf = build_standard_form(tableau.c, tableau.rows, bool(maximize))
    res = solve_standard_form(sf, device=device, rule=rule, max_iters=max_iters,
                              time_limit=time_limit, record=True,
                              cell_budget=HISTORY_CELL_BUDGET)
    out = {
        "pivotSteps": res.steps,
        "status": STATUS_TEXT.get(res.status, str(res.status)),
        "status_code": res.status,
        "iterations": res.iters,
        "objective": res.objective,
        "solution": (None if res.x is None
                     else {f"x{i + 1}": float(v) for i, v in enumerate(res.x)}),
        "basis": None if res.basis is None else [int(b) for b in res.basis],
    }
    return out
