"""Generate the committed golden fixtures under tests/golden/.

Run from the repo root:  python tests/golden/make_golden.py

textbook.json
  The LPs of the reference's own tests (cited per case) plus the classic Beale
  cycling LP, each with: the oracle's pivot sequences (Dantzig, Bland), final
  basis, status, objective and x; HiGHS (scipy linprog 'highs-ds', the
  reference's answer path, solver_controller.py:76-85) status/objective; and
  the reference test's stated answer where it is a true optimum.  The script
  asserts oracle == HiGHS == reference answer before writing.
pivots.npz / pivots_sha256.json
  Seeded random tableaux (odd sizes, ties, zero columns, negative entries)
  with the oracle's result after one pivot: the bit-exact single-pivot
  vectors for the elimination kernel.
dense_lp.json
  Generated dense LPs (simplex_amd.synth generator) with HiGHS objective and
  the oracle's pivot count / objective, for solve-level parity.
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np
from scipy.optimize import linprog

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "simplex-solver_amd"))

from oracle import simplex_oracle as O  # noqa: E402
from simplex_amd import synth  # noqa: E402

REF = "/root/reference/"  # cited paths, relative to the reference root

TEXTBOOK = [
    dict(name="max_15_18", cite="tests/test_solver_controller.py:32-46", maximize=True,
         c=[15, 18], rows=[([4, 2], "<=", 2000), ([2, 6], "<=", 2400), ([20, 28], "<=", 14000)],
         ref_answer=dict(z=9833.333333333334, x=[388.8888888888889, 222.22222222222223])),
    dict(name="wyndor", cite="tests/test_visualization_integration.py:38-56", maximize=True,
         c=[3, 5], rows=[([1, 0], "<=", 4), ([0, 2], "<=", 12), ([3, 2], "<=", 18)],
         ref_answer=dict(z=36.0, x=[2.0, 6.0])),
    # the reference test holds Z = 30 only; its mocked x = (5, 3, 2) is not an
    # optimum (:447-452), so x is HiGHS's, kept apart as highs_x
    dict(name="three_var", cite="tests/test_visualization_integration.py:417-444 (config 1)",
         maximize=True, c=[1, 2, 3],
         rows=[([1, 1, 1], "<=", 10), ([2, 1, 0], "<=", 15), ([0, 2, 1], "<=", 12)],
         ref_answer=dict(z=30.0), highs_x=[0.0, 0.0, 10.0]),
    dict(name="equality", cite="tests/test_visualization_integration.py:205-224", maximize=True,
         c=[1, 1], rows=[([1, 1], "=", 10), ([2, 1], "<=", 15)], ref_answer=dict(z=10.0)),
    dict(name="infeasible", cite="tests/test_visualization_integration.py:240-259",
         maximize=True, c=[1], rows=[([1], "<=", 5), ([1], ">=", 10)],
         ref_answer=dict(status=2)),
    dict(name="no_constraints", cite="tests/test_visualization_integration.py:346-362",
         maximize=True, c=[1, 1], rows=[], ref_answer=dict(status=3)),
    dict(name="zero_coef", cite="tests/test_visualization_integration.py:375-395",
         maximize=True, c=[0, 5], rows=[([1, 0], "<=", 10), ([0, 1], "<=", 5)],
         ref_answer=dict(z=25.0, x=[0.0, 5.0])),
    dict(name="min_50_80", cite="tests/test_solver_controller.py:16-30 (mocked answer is NOT "
         "an optimum; true optimum from HiGHS)", maximize=False, c=[50, 80],
         rows=[([4, 1], ">=", 4), ([1, 6], ">=", 6), ([4, 6], ">=", 12)], ref_answer=None),
    dict(name="min_2_3", cite="tests/test_visualization_integration.py:59-75 (mocked answer is "
         "NOT an optimum)", maximize=False, c=[2, 3],
         rows=[([1, 1], ">=", 5), ([2, 1], ">=", 8)], ref_answer=None),
    dict(name="ui_mock", cite="tests/test_ui_controller.py:28-41", maximize=True, c=[1, 2],
         rows=[([1, 1], "<=", 10)], ref_answer=dict(z=20.0, x=[0.0, 10.0])),
    dict(name="beale", cite="Beale (1955) cycling example; SURVEY.md §8c", maximize=True,
         c=[0.75, -20, 0.5, -6],
         rows=[([0.25, -8, -1, 9], "<=", 0), ([0.5, -12, -0.5, 3], "<=", 0),
               ([0, 0, 1, 0], "<=", 1)], ref_answer=dict(z=1.25)),
    dict(name="negative_rhs", cite="build spec: b < 0 rows are negated (DESIGN.md §2)",
         maximize=False, c=[1, 1], rows=[([-1, -2], "<=", -4), ([3, 1], "<=", 9)],
         ref_answer=None),
    dict(name="unbounded", cite="build spec: unbounded ray", maximize=True, c=[1, 1],
         rows=[([1, -1], "<=", 1)], ref_answer=dict(status=3)),
]

HIGHS_STATUS = {0: 0, 1: 1, 2: 2, 3: 3, 4: 4}


def highs(case):
    c = np.array(case["c"], dtype=float)
    A_ub, b_ub, A_eq, b_eq = [], [], [], []
    for a, op, b in case["rows"]:
        if op == "<=":
            A_ub.append(a); b_ub.append(b)
        elif op == ">=":
            A_ub.append([-x for x in a]); b_ub.append(-b)
        else:
            A_eq.append(a); b_eq.append(b)
    res = linprog(-c if case["maximize"] else c, A_ub=A_ub or None, b_ub=b_ub or None,
                  A_eq=A_eq or None, b_eq=b_eq or None, bounds=[(0, None)] * len(c),
                  method="highs-ds")
    z = None
    if res.status == 0:
        z = float(-res.fun if case["maximize"] else res.fun)
    return int(res.status), z


def textbook():
    out = []
    for case in TEXTBOOK:
        entry = dict(name=case["name"], cite=case["cite"], maximize=case["maximize"],
                     c=case["c"], rows=[[list(map(float, a)), op, float(b)]
                                        for a, op, b in case["rows"]])
        hs, hz = highs(case)
        entry["highs"] = dict(status=hs, objective=hz)
        for rule in ("dantzig", "bland"):
            r = O.solve_lp(case["c"], case["rows"], case["maximize"], rule=rule, max_iters=200)
            entry[rule] = dict(status=r["status"],
                               objective=r["objective"],
                               x=None if r["x"] is None else r["x"].tolist(),
                               pivots=[list(p) for p in r["pivots"]],
                               basis=r["basis"].tolist(),
                               final_tableau=r["T"].tolist())
        # cross-checks before writing
        bl = entry["bland"]
        assert bl["status"] == hs, (case["name"], bl["status"], hs)
        if hs == 0:
            assert abs(bl["objective"] - hz) <= 1e-9 * max(1.0, abs(hz)), case["name"]
        ref = case["ref_answer"]
        if ref:
            if "z" in ref:
                assert abs(bl["objective"] - ref["z"]) <= 1e-9 * max(1, abs(ref["z"])), case
            if "status" in ref:
                assert bl["status"] == ref["status"], case["name"]
        entry["ref_answer"] = ref
        if "highs_x" in case:  # an x from HiGHS, not from the reference tests
            entry["highs"]["x"] = case["highs_x"]
        out.append(entry)
    return out


PIVOT_SHAPES = [(1, 2), (3, 5), (7, 12), (33, 70), (130, 257), (513, 1100), (1025, 3073)]
FULL_ARRAY_CELLS = 40_000  # larger cases are pinned by SHA-256 of the result bytes


def pivot_case(k):
    """Deterministic single-pivot input k (also regenerated by the tests)."""
    rows, cols = PIVOT_SHAPES[k]
    rng = np.random.default_rng(20251205 + k)
    T = rng.uniform(-2, 2, size=(rows, cols))
    # exact zeros in the pivot row and elsewhere, integer ties
    T[rng.random((rows, cols)) < 0.2] = 0.0
    if rows > 2:
        T[:rows // 2, : cols // 3] = np.round(T[:rows // 2, : cols // 3])
    m = rows - 1
    r = int(rng.integers(0, max(m, 1))) if m else 0
    c = int(rng.integers(0, cols - 1))
    if m:
        T[r, c] = 1.5 if T[r, c] == 0 else abs(T[r, c]) + 0.25
    return T, r, c


def pivot_vectors():
    import hashlib
    arrays, digests = {}, {}
    for k in range(len(PIVOT_SHAPES)):
        T, r, c = pivot_case(k)
        for skip in (True, False):
            after = T.copy()
            if T.shape[0] > 1:
                O.pivot(after, r, c, skip_zero=skip)
            tag = f"case{k}_after_{'skip' if skip else 'dense'}"
            digests[tag] = hashlib.sha256(np.ascontiguousarray(after).tobytes()).hexdigest()
            if T.size <= FULL_ARRAY_CELLS:
                arrays[tag] = after
        if T.size <= FULL_ARRAY_CELLS:
            arrays[f"case{k}_T"] = T
        arrays[f"case{k}_rc"] = np.array([r, c], dtype=np.int64)
    arrays["ncases"] = np.array([len(PIVOT_SHAPES)])
    return arrays, digests


def dense_lps():
    out = []
    for (m, n, seed) in [(16, 24, 1), (64, 96, 7), (200, 300, 11), (1024, 2048, 20251207)]:
        A, b, c = synth.lp_data("dense", m, n, seed)
        res = linprog(-c, A_ub=A, b_ub=b, bounds=[(0, None)] * n, method="highs-ds")
        T, basis = synth.full_tableau("dense", m, n, seed)
        st, hist = O.solve_tableau(T, basis)
        assert st == 0 and abs(T[-1, -1] + res.fun) <= 1e-9 * abs(res.fun), (m, n)
        out.append(dict(m=m, n=n, seed=seed, kind="dense", highs_objective=float(-res.fun),
                        highs_nit=int(res.nit), oracle_objective=float(T[-1, -1]),
                        oracle_pivots=len(hist), oracle_first_pivots=[list(h) for h in hist[:32]],
                        oracle_final_basis_head=basis[:64].tolist()))
    for (m, n, seed) in [(64, 64, 5), (128, 128, 5)]:
        A, b, c = synth.lp_data("degenerate", m, n, seed)
        res = linprog(-c, A_ub=A, b_ub=b, bounds=[(0, None)] * n, method="highs-ds")
        T, basis = synth.full_tableau("degenerate", m, n, seed)
        st, hist = O.solve_tableau(T, basis, rule="bland", max_iters=100000)
        assert st == 0 and abs(T[-1, -1] + res.fun) <= 1e-9 * max(1, abs(res.fun)), (m, n)
        out.append(dict(m=m, n=n, seed=seed, kind="degenerate", rule="bland",
                        highs_objective=float(-res.fun), highs_nit=int(res.nit),
                        oracle_objective=float(T[-1, -1]), oracle_pivots=len(hist),
                        oracle_first_pivots=[list(h) for h in hist[:32]]))
    return out


if __name__ == "__main__":
    with open(os.path.join(HERE, "textbook.json"), "w") as f:
        json.dump(textbook(), f, indent=1)
    arrays, digests = pivot_vectors()
    np.savez_compressed(os.path.join(HERE, "pivots.npz"), **arrays)
    with open(os.path.join(HERE, "pivots_sha256.json"), "w") as f:
        json.dump(digests, f, indent=1)
    with open(os.path.join(HERE, "dense_lp.json"), "w") as f:
        json.dump(dense_lps(), f, indent=1)
    print("golden fixtures written")
