"""The CPU oracle against the committed golden vectors (no GPU).

Pins: the reference tests' known answers and HiGHS (both recorded in
tests/golden/textbook.json by make_golden.py, which asserted them), plus the
oracle's own pivot sequences / final tableaux, so that any change to the
oracle is caught before it is used as the checker of the HIP path.
"""
import hashlib
import json
import os

import numpy as np
import pytest

from oracle import simplex_oracle as O

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
TEXTBOOK = json.load(open(os.path.join(HERE, "textbook.json")))
DENSE = json.load(open(os.path.join(HERE, "dense_lp.json")))


def _rows(e):
    return [(a, op, b) for a, op, b in e["rows"]]


@pytest.mark.parametrize("case", TEXTBOOK, ids=[e["name"] for e in TEXTBOOK])
@pytest.mark.parametrize("rule", ["dantzig", "bland"])
def test_textbook_oracle_matches_golden(case, rule):
    r = O.solve_lp(case["c"], _rows(case), case["maximize"], rule=rule, max_iters=200)
    g = case[rule]
    assert r["status"] == g["status"]
    assert [list(p) for p in r["pivots"]] == g["pivots"]
    assert r["basis"].tolist() == g["basis"]
    assert np.array_equal(r["T"], np.array(g["final_tableau"]))
    if g["status"] == 0:
        assert r["objective"] == g["objective"]


@pytest.mark.parametrize("case", TEXTBOOK, ids=[e["name"] for e in TEXTBOOK])
def test_textbook_answers_pinned_to_highs_and_reference(case):
    g = case["bland"]
    assert g["status"] == case["highs"]["status"]
    if g["status"] == 0:
        hz = case["highs"]["objective"]
        assert abs(g["objective"] - hz) <= 1e-9 * max(1.0, abs(hz))
    ref = case["ref_answer"]
    if ref and "z" in ref:
        assert abs(g["objective"] - ref["z"]) <= 1e-9 * max(1.0, abs(ref["z"]))
    if ref and "x" in ref and case["name"] != "equality":
        assert np.allclose(g["x"], ref["x"], rtol=1e-9, atol=1e-9)
    if ref and "status" in ref:
        assert g["status"] == ref["status"]


def test_survey_pivot_sequences():
    """SURVEY.md §8c golden sequences (layout [A|I|b], objective row last)."""
    by = {e["name"]: e for e in TEXTBOOK}
    seq = lambda e, rule: [tuple(p[1:]) for p in e[rule]["pivots"]]  # noqa: E731
    assert seq(by["wyndor"], "dantzig") == [(1, 1), (2, 0)]
    assert by["wyndor"]["dantzig"]["basis"] == [2, 1, 0]
    assert seq(by["wyndor"], "bland") == [(0, 0), (2, 1), (1, 2)]
    assert seq(by["max_15_18"], "dantzig") == [(1, 1), (2, 0), (0, 3)]
    assert seq(by["max_15_18"], "bland") == [(0, 0), (2, 1)]
    assert seq(by["three_var"], "dantzig") == [(0, 2)]
    assert len(seq(by["three_var"], "bland")) == 5
    # Beale: Dantzig with lowest-index ties cycles with period 6, Bland ends in 6
    d = seq(by["beale"], "dantzig")
    assert by["beale"]["dantzig"]["status"] == O.ITER_LIMIT and d[:6] == d[6:12]
    assert len(seq(by["beale"], "bland")) == 6
    assert abs(by["beale"]["bland"]["objective"] - 1.25) < 1e-12


def _pivot_case(k):
    import importlib.util
    spec = importlib.util.spec_from_file_location("make_golden", os.path.join(HERE,
                                                                              "make_golden.py"))
    mg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mg)
    return mg.pivot_case(k), mg


def test_single_pivot_vectors():
    z = np.load(os.path.join(HERE, "pivots.npz"))
    digests = json.load(open(os.path.join(HERE, "pivots_sha256.json")))
    n = int(z["ncases"][0])
    for k in range(n):
        (T, r, c), _ = _pivot_case(k)
        assert z[f"case{k}_rc"].tolist() == [r, c]
        if f"case{k}_T" in z:
            assert np.array_equal(z[f"case{k}_T"], T)
        for tag in ("skip", "dense"):
            after = T.copy()
            if T.shape[0] > 1:
                O.pivot(after, r, c, skip_zero=(tag == "skip"))
            key = f"case{k}_after_{tag}"
            assert hashlib.sha256(after.tobytes()).hexdigest() == digests[key]
            if key in z:
                assert np.array_equal(z[key], after)


def test_skip_rule_equals_dense_update_up_to_zero_sign():
    rng = np.random.default_rng(3)
    for _ in range(20):
        T = rng.uniform(-3, 3, size=(9, 14))
        T[rng.random(T.shape) < 0.3] = 0.0
        r, c = int(rng.integers(0, 8)), int(rng.integers(0, 13))
        T[r, c] = 2.0
        a, b = T.copy(), T.copy()
        O.pivot(a, r, c, skip_zero=True)
        O.pivot(b, r, c, skip_zero=False)
        assert np.array_equal(a, b)  # == treats -0.0 and +0.0 as equal


@pytest.mark.parametrize("e", [e for e in DENSE if e["m"] <= 200],
                         ids=lambda e: f"{e['kind']}{e['m']}x{e['n']}")
def test_generated_lps_oracle_vs_highs(e):
    import sys
    from simplex_amd import synth
    T, basis = synth.full_tableau(e["kind"], e["m"], e["n"], e["seed"])
    rule = e.get("rule", "dantzig")
    st, hist = O.solve_tableau(T, basis, rule=rule, max_iters=200000)
    assert st == 0
    assert len(hist) == e["oracle_pivots"]
    assert [list(h) for h in hist[:32]] == e["oracle_first_pivots"]
    assert T[-1, -1] == e["oracle_objective"]
    hz = e["highs_objective"]
    assert abs(T[-1, -1] - hz) <= 1e-9 * max(1.0, abs(hz))


@pytest.mark.parametrize("kind,m,n,seed,rule", [("dense", 64, 96, 7, "dantzig"),
                                                 ("dense", 200, 300, 11, "dantzig"),
                                                 ("degenerate", 64, 64, 5, "bland")])
@pytest.mark.parametrize("skip", [True, False])
def test_c_oracle_bit_identical_to_numpy_oracle(kind, m, n, seed, rule, skip):
    from oracle import c_oracle as C
    from simplex_amd import synth
    T, b = synth.full_tableau(kind, m, n, seed)
    T2, b2 = T.copy(), b.copy()
    st, h = O.solve_tableau(T, b, rule=rule, max_iters=100000, skip_zero=skip)
    st2, h2 = C.solve(T2, b2, rule=rule, skip_zero=skip)
    assert st == st2 and h == h2 and np.array_equal(b, b2)
    assert T.tobytes() == T2.tobytes()


# ----------------------------------------------------------- full-size fixtures
def _fullsize():
    import json
    import os
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "fullsize.json")
    if not os.path.exists(path):
        pytest.skip("fullsize.json not generated")
    return json.load(open(path))


def test_fullsize_fixtures_consistent_with_highs_and_acyclic():
    """The oracle's full-size runs (tests/golden/make_fullsize.py) agree with
    HiGHS (the reference's answer path, solver_controller.py:76-85) within
    1e-9 wherever they reached optimality, and revisit no basis."""
    import os
    fx = _fullsize()
    here = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    for name, f in fx.items():
        if "pivots" not in f:
            continue
        z = np.load(os.path.join(here, f"fullsize_{name}.npz"))
        assert z["hist"].shape == (f["pivots"], 2)
        assert f.get("basis_repeats", 0) == 0
        if f["status"] == 0 and f.get("highs_status") == 0:
            hz = f["highs_objective"]
            assert abs(f["objective"] - hz) <= 1e-9 * max(1.0, abs(hz)), name
            assert float.fromhex(f["objective_hex"]) == f["objective"]


def test_zobrist_detects_a_revisited_basis():
    """The cycle detector itself: Beale's LP under Dantzig revisits its first
    basis after 6 pivots."""
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
    from make_fullsize import zobrist_repeats
    sf = O.standard_form([0.75, -20, 0.5, -6],
                         [([0.25, -8, -1, 9], "<=", 0), ([0.5, -12, -0.5, 3], "<=", 0),
                          ([0, 0, 1, 0], "<=", 1)], True)
    T, b = sf["T"], sf["basis"].copy()
    b0 = b.copy()
    st, h = O.solve_tableau(T, b, rule="dantzig", max_iters=12)
    assert st == 1 and zobrist_repeats(np.asarray(h, dtype=np.int64), b0) > 0
