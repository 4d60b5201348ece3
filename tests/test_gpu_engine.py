"""Parity of the HIP pivot engine (through the C-ABI) with the CPU oracle.

Bar: bit-exact tableaux, pivot sequences and bases (np.array_equal, which
treats -0.0 == +0.0); objectives additionally within 1e-9 relative of HiGHS.
"""
import hashlib
import importlib.util
import json
import os
import threading

import numpy as np
import pytest

from oracle import simplex_oracle as O

pytestmark = pytest.mark.gpu

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
TEXTBOOK = json.load(open(os.path.join(HERE, "textbook.json")))
DENSE = json.load(open(os.path.join(HERE, "dense_lp.json")))


def _mg():
    spec = importlib.util.spec_from_file_location("make_golden",
                                                  os.path.join(HERE, "make_golden.py"))
    mg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mg)
    return mg


@pytest.fixture(scope="module")
def eng_cls():
    from simplex_amd.engine import DeviceTableau
    return DeviceTableau


def _rows(e):
    return [(a, op, b) for a, op, b in e["rows"]]


# ----------------------------------------------------------- single pivots
def test_single_pivot_vectors_bit_exact(eng_cls):
    """spx_pivot_at on the golden single-pivot inputs (tests/golden/pivots*)."""
    mg = _mg()
    digests = json.load(open(os.path.join(HERE, "pivots_sha256.json")))
    for k in range(len(mg.PIVOT_SHAPES)):
        T, r, c = mg.pivot_case(k)
        if T.shape[0] < 2:
            continue
        basis = np.arange(T.shape[0] - 1, dtype=np.int64)
        with eng_cls(0) as e:
            e.load(T, basis)
            e.pivot_at(r, c)
            out = e.tableau()
        ref = T.copy()
        O.pivot(ref, r, c, skip_zero=True)
        assert np.array_equal(out, ref), f"case {k}"
        assert hashlib.sha256(ref.tobytes()).hexdigest() == digests[f"case{k}_after_skip"]
        # bit-level: the only allowed difference is none at all here
        assert out.tobytes() == ref.tobytes(), f"case {k}: not bitwise identical"


@pytest.mark.parametrize("shape", [(2, 3), (17, 40), (300, 700), (1025, 2051), (2049, 4097)])
@pytest.mark.parametrize("skip", [True, False], ids=["skip", "dense"])
def test_rule_pivots_bit_exact_random(eng_cls, shape, skip):
    """Rule-chosen pivots on random feasible tableaux: sequence + bits."""
    rows, cols = shape
    rng = np.random.default_rng(rows * 7 + cols)
    m = rows - 1
    n = cols - 1 - m
    if n < 1:
        n = 1
    A = rng.uniform(0.05, 1.0, size=(m, n))
    A[rng.random(A.shape) < 0.1] = 0.0
    T = np.zeros((m + 1, n + m + 1))
    T[:m, :n] = A
    T[np.arange(m), n + np.arange(m)] = 1.0
    T[:m, -1] = rng.uniform(1, 2, size=m) * n
    T[m, :n] = -rng.uniform(0.1, 1, size=n)
    basis = np.arange(n, n + m, dtype=np.int64)
    ref, rb = T.copy(), basis.copy()
    st, hist = O.solve_tableau(ref, rb, max_iters=12, skip_zero=skip)
    with eng_cls(0) as e:
        e.load(T, basis)
        res = e.solve(max_iters=12, skip_zero_cols=skip)
        assert [tuple(h) for h in e.history().tolist()] == hist
        assert np.array_equal(e.tableau(), ref)
        assert np.array_equal(e.basis(), rb)
        assert res.status == st


# ----------------------------------------------------------- textbook LPs
@pytest.mark.parametrize("case", TEXTBOOK, ids=[e["name"] for e in TEXTBOOK])
@pytest.mark.parametrize("rule", ["dantzig", "bland"])
def test_textbook_through_simple_simplex(case, rule):
    from simplex_amd import simple_simplex as ss
    n = len(case["c"])
    t = ss.create_tableau(number_of_variables=n, number_of_constraints=len(case["rows"]))
    for a, op, b in case["rows"]:
        code = {"<=": "L", ">=": "G", "=": "E"}[op]
        t_str = ",".join(str(x) for x in a) + f",{code},{b}"
        ss.add_constraint(t, t_str)
    ss.add_objective(t, ",".join(str(x) for x in case["c"]) + (",1" if case["maximize"] else ",0"))
    out = ss.optimize_json_format(t, maximize=case["maximize"], rule=rule, max_iters=200)
    g = case[rule]
    assert out["status_code"] == g["status"]
    steps = out["pivotSteps"]
    got = [[s["phase"], s["pivotRowIndex"], s["pivotColIndex"]] for s in steps
           if s["pivotRowIndex"] is not None]
    assert got == g["pivots"]
    assert out["basis"] == g["basis"]
    assert np.array_equal(np.array(steps[-1]["tableau"]), np.array(g["final_tableau"]))
    if g["status"] == 0:
        assert out["objective"] == g["objective"]
        hz = case["highs"]["objective"]
        assert abs(out["objective"] - hz) <= 1e-9 * max(1, abs(hz))
    # every recorded snapshot equals the oracle replayed to that step
    r = O.standard_form(case["c"], _rows(case), case["maximize"])
    assert np.array_equal(np.array(steps[0]["tableau"]), r["T"])


# ----------------------------------------------------------- generated LPs
@pytest.mark.parametrize("e", DENSE, ids=lambda e: f"{e['kind']}{e['m']}x{e['n']}")
def test_generated_lp_full_solve(eng_cls, e):
    from simplex_amd import synth
    T, basis = synth.full_tableau(e["kind"], e["m"], e["n"], e["seed"])
    rule = e.get("rule", "dantzig")
    with eng_cls(0) as eng:
        eng.load(T, basis)
        res = eng.solve(rule=rule)
        hist = eng.history()
        assert res.status == 0
        assert len(hist) == e["oracle_pivots"]
        assert hist[:32].tolist() == e["oracle_first_pivots"]
        assert res.objective == e["oracle_objective"]
        hz = e["highs_objective"]
        assert abs(res.objective - hz) <= 1e-9 * max(1.0, abs(hz))
        if e["m"] <= 256:
            ref, rb = T.copy(), basis.copy()
            O.solve_tableau(ref, rb, rule=rule, max_iters=200000)
            assert np.array_equal(eng.tableau(), ref)
            assert np.array_equal(eng.basis(), rb)


def test_config2_full_history_matches_oracle(eng_cls):
    """1024x2048 random feasible LP (BASELINE config 2): every pivot index."""
    from simplex_amd import synth
    e = [d for d in DENSE if d["m"] == 1024][0]
    T, basis = synth.full_tableau("dense", 1024, 2048, e["seed"])
    ref, rb = T.copy(), basis.copy()
    st, hist = O.solve_tableau(ref, rb)
    with eng_cls(0) as eng:
        eng.load(T, basis)
        res = eng.solve()
        assert [tuple(h) for h in eng.history().tolist()] == hist
        assert np.array_equal(eng.basis(), rb)
        assert np.array_equal(eng.tableau(), ref)
        assert res.objective == ref[-1, -1]


def test_degenerate_bland_every_pivot(eng_cls):
    from simplex_amd import synth
    T, basis = synth.full_tableau("degenerate", 96, 96, 9)
    ref, rb = T.copy(), basis.copy()
    seen = []
    st, hist = O.solve_tableau(ref, rb, rule="bland", max_iters=100000,
                               on_pivot=lambda r, c, _T: seen.append(rb.copy()))
    assert st == 0
    with eng_cls(0) as eng:
        eng.load(T, basis)
        # step through, checking the basis after every pivot
        for k in range(min(60, len(hist))):
            out = eng.pivot(rule="bland")
            assert out == hist[k]
            assert np.array_equal(eng.basis(), seen[k])
        res = eng.solve(rule="bland")
        assert res.status == 0
        assert [tuple(h) for h in eng.history().tolist()] == hist
        assert np.array_equal(eng.tableau(), ref)


# ----------------------------------------------------------- modes, edges
def test_graph_and_direct_and_chunks_agree(eng_cls):
    from simplex_amd import synth
    T, basis = synth.full_tableau("dense", 200, 300, 11)
    outs = []
    # (single-pivot solves ramp their chunks 4, 8, 16, ... up to `chunk`, then
    # replay its graph: chunk 100 ramps through 64 first)
    for kw in (dict(use_graph=True, chunk=32), dict(use_graph=False, chunk=8),
               dict(use_graph=True, chunk=1), dict(use_graph=True, chunk=7),
               dict(use_graph=True, chunk=100), dict(use_graph=False, chunk=100)):
        with eng_cls(0) as eng:
            eng.load(T, basis)
            res = eng.solve(**kw)
            outs.append((res.status, res.iters, eng.history().tolist(), eng.tableau()))
    for o in outs[1:]:
        assert o[0] == outs[0][0] and o[1] == outs[0][1] and o[2] == outs[0][2]
        assert np.array_equal(o[3], outs[0][3])


def test_reload_same_shape_keeps_buffers_bit_exact(eng_cls):
    """One context, many loads (round 6: a reload of the loaded shape keeps the
    device buffers and only clears them, the pooled contexts of the user
    path).  LPs of one shape with other seeds, both rules, windows of 8 and 24
    and single pivots, an unfinished solve before each reload (its window
    state, records and history must not leak into the next load), another
    shape in between and back: every run equals the oracle's run from its own
    load."""
    from simplex_amd import synth
    shapes = [(120, 200, 1, "dense"), (120, 200, 2, "dense"), (120, 200, 3, "degenerate"),
              (64, 100, 4, "dense"), (120, 200, 5, "degenerate"), (120, 200, 6, "dense"),
              (700, 900, 7, "dense"), (700, 900, 8, "dense")]
    with eng_cls(0) as eng:
        for k, (m, n, seed, kind) in enumerate(shapes):
            rule = "bland" if kind == "degenerate" else "dantzig"
            T, basis = synth.full_tableau(kind, m, n, seed)
            ref, rb = T.copy(), basis.copy()
            st, hist = O.solve_tableau(ref, rb, rule=rule, max_iters=3000)
            window = (0, 8, 24)[k % 3]
            # an unfinished windowed solve of the same data first, then the reload
            eng.set_window(16)
            eng.load(T, basis)
            eng.solve(rule=rule, max_iters=37)
            eng.set_window(window)
            eng.load(T, basis)
            for q in range(min(3, len(hist))):
                assert eng.pivot(rule=rule) == hist[q]
            res = eng.solve(rule=rule, max_iters=3000 - min(3, len(hist)))
            assert res.status == st, (k, res.status, st)
            assert [tuple(h) for h in eng.history().tolist()] == hist, k
            assert np.array_equal(eng.tableau(), ref), k
            assert np.array_equal(eng.basis(), rb), k
        eng.set_window(0)


def test_iteration_limit_and_resume(eng_cls):
    from simplex_amd import synth
    T, basis = synth.full_tableau("dense", 64, 96, 7)
    with eng_cls(0) as a, eng_cls(0) as b:
        a.load(T, basis)
        b.load(T, basis)
        r1 = a.solve(max_iters=5)
        assert r1.status == 1 and r1.iters == 5
        r2 = a.solve()
        rb = b.solve()
        assert r2.status == rb.status == 0 and r1.iters + r2.iters == rb.iters
        assert a.history().tolist() == b.history().tolist()
        assert np.array_equal(a.tableau(), b.tableau())


def test_beale_cycles_under_dantzig_and_bland_terminates(eng_cls):
    from simplex_amd import lp
    c = [0.75, -20, 0.5, -6]
    rows = [([0.25, -8, -1, 9], "<=", 0), ([0.5, -12, -0.5, 3], "<=", 0),
            ([0, 0, 1, 0], "<=", 1)]
    sf = lp.build_standard_form(c, rows, True)
    with eng_cls(0) as e:
        e.load(sf.T, sf.basis)
        res = e.solve(max_iters=60)
        h = e.history().tolist()
        assert res.status == 1 and h[:6] == h[6:12]
    res = lp.solve_lp(c, rows, True, rule="bland")
    assert res.status == 0 and abs(res.objective - 1.25) < 1e-12 and res.iters == 6


def test_edges(eng_cls):
    # no constraints: any improving column is unbounded
    with eng_cls(0) as e:
        e.load(np.array([[-1.0, -2.0, 0.0]]), np.zeros(0, dtype=np.int64))
        assert e.solve().status == 3
    # already optimal
    with eng_cls(0) as e:
        e.load(np.array([[1.0, 1.0, 0.0, 4.0], [1.0, 0.0, 0.0, 0.0]]), np.array([2]))
        r = e.solve()
        assert r.status == 0 and r.iters == 0
    # unbounded column
    with eng_cls(0) as e:
        e.load(np.array([[-1.0, 1.0, 1.0, 1.0], [-1.0, -1.0, 0.0, 0.0]]), np.array([2]))
        assert e.solve().status == 3


def test_concurrent_contexts_from_threads(eng_cls):
    """/solve is entered from many threads (reference test_performance_load.py:80-83)."""
    from simplex_amd import synth
    cases = [(40 + 9 * k, 60 + 7 * k, k) for k in range(6)]
    errors, results = [], {}

    def work(m, n, s):
        try:
            T, basis = synth.full_tableau("dense", m, n, s)
            with eng_cls(0) as e:
                e.load(T, basis)
                results[s] = (e.solve().objective, e.history().tolist())
        except Exception as ex:  # pragma: no cover
            errors.append(ex)

    th = [threading.Thread(target=work, args=c) for c in cases]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors
    for m, n, s in cases:
        T, basis = synth.full_tableau("dense", m, n, s)
        st, hist = O.solve_tableau(T, basis)
        assert results[s][0] == T[-1, -1] and [tuple(h) for h in results[s][1]] == hist


def test_sharded_single_rank_matches_plain(eng_cls):
    """RCCL communicator of one rank: exercises the sharded kernels
    (select / all-gather / PROW / all-reduce / FINISH) end to end."""
    from simplex_amd import dist, synth
    T, basis = synth.full_tableau("dense", 200, 300, 11)
    ref, rb = T.copy(), basis.copy()
    st, hist = O.solve_tableau(ref, rb)
    uid = dist.make_unique_id()
    with dist.ShardedTableau(0, 0, 1, uid) as s:
        s.load_shard(T[:-1], T[-1], basis, 200, 0)
        res = s.solve()
        assert res.status == 0
        assert [tuple(h) for h in s.history().tolist()] == hist
        assert np.array_equal(s.tableau(), ref)


# ----------------------------------------------------------- full size
def test_config3_size_first_pivots_bit_exact(eng_cls):
    """8192 x 16385 tableau (BASELINE config 3): first pivots vs oracle, then
    size-independent invariants over further pivots."""
    from simplex_amd import synth
    m = n = 8192
    Tf, obj, basis = synth.tableau_rows("dense", m, n, 20251205, order="F")
    with eng_cls(0) as e:
        e.load_rows(Tf, obj, basis, m, 0)
        T = np.vstack([np.ascontiguousarray(Tf), obj[None, :]])
        del Tf
        rb = basis.copy()
        st, hist = O.solve_tableau(T, rb, max_iters=3)
        res = e.solve(max_iters=3)
        assert [tuple(h) for h in e.history().tolist()] == hist
        assert np.array_equal(e.tableau(), T)
        del T
        z_prev = e.objective_row()[-1]
        res = e.solve(max_iters=40)
        assert res.status == 1 and res.iters == 40
        b = e.basis()
        assert len(set(b.tolist())) == m
        objrow = e.objective_row()
        assert objrow[-1] >= z_prev  # Dantzig from a feasible basis never decreases Z
        assert np.all(objrow[b] == 0.0)
        for k in np.random.default_rng(0).choice(m, 16, replace=False):
            col = e.column(int(b[k]))
            assert col[k] == 1.0 and np.count_nonzero(col) == 1  # basic columns = e_k
        assert e.column(m + n).min() >= -1e-9  # RHS stays feasible


# ----------------------------------------------------------- sharded, nranks > 1
def _sharded_threads(world, kind, m, n, seed, rule, window=0, **solve_kw):
    from simplex_amd import dist, synth
    uid = bytes([world, m % 251, n % 251, seed % 251]) + os.urandom(124)
    outs, errors = {}, []

    def rank_main(rank):
        try:
            r0, r1 = dist.row_partition(m, world, rank)
            T, obj, basis = synth.tableau_rows(kind, m, n, seed, r0, r1, order="F")
            with dist.ShardedTableau(0, rank, world, uid, local=True) as s:
                s.set_window(window)
                s.load_shard(T, obj, basis, m, r0)
                res = s.solve(rule=rule, **solve_kw)
                outs[rank] = (r0, r1, res, s.history().tolist(), s.tableau(), s.basis())
        except Exception as ex:  # pragma: no cover
            errors.append(ex)

    th = [threading.Thread(target=rank_main, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=600)
    assert not errors, errors
    return outs


@pytest.mark.parametrize("world,kind,m,n,rule", [
    (2, "dense", 200, 300, "dantzig"),
    (3, "dense", 301, 257, "dantzig"),
    (4, "dense", 1024, 2048, "dantzig"),
    (2, "degenerate", 64, 64, "bland"),
    (5, "dense", 7, 9, "dantzig"),   # ranks with one or two rows
])
def test_sharded_virtual_ranks_bit_exact(world, kind, m, n, rule):
    """nranks > 1 sharded kernels (select / PROW / FINISH, row offsets,
    owner vs non-owner ranks) on one GPU through the in-process exchange."""
    from simplex_amd import synth
    outs = _sharded_threads(world, kind, m, n, 3, rule)
    T, basis = synth.full_tableau(kind, m, n, 3)
    st, hist = O.solve_tableau(T, basis, rule=rule, max_iters=200000)
    for rank, (r0, r1, res, h, Tl, b) in outs.items():
        assert res.status == st
        assert [tuple(x) for x in h] == hist
        assert np.array_equal(Tl[:-1], T[r0:r1])
        assert np.array_equal(Tl[-1], T[-1])
        assert np.array_equal(b, basis)


@pytest.mark.parametrize("window", [0, 8])
def test_sharded_time_limit_stops_every_rank_at_one_pivot(window):
    """time_limit on row shards (the reference always passes time_limit 10,
    solver_controller.py:76): rank 0's host asks its device to stop, its
    payload header carries the request, and every rank stops before the same
    pivot with status 1 (iteration / time limit), bit-exact to the oracle
    after that many pivots."""
    from simplex_amd import synth
    m, n = 600, 900
    outs = _sharded_threads(3, "dense", m, n, 5, "dantzig", window=window, time_limit=1e-4)
    T, basis = synth.full_tableau("dense", m, n, 5)
    _, full = O.solve_tableau(T.copy(), basis.copy(), max_iters=200000)
    iters = {res.iters for (_, _, res, _, _, _) in outs.values()}
    hists = {tuple(map(tuple, h)) for (_, _, _, h, _, _) in outs.values()}
    assert len(iters) == 1 and len(hists) == 1
    k = iters.pop()
    assert 0 < k < len(full)
    st, hist = O.solve_tableau(T, basis, max_iters=k)
    for rank, (r0, r1, res, h, Tl, b) in outs.items():
        assert res.status == 1
        assert [tuple(x) for x in h] == hist
        assert np.array_equal(Tl[:-1], T[r0:r1]) and np.array_equal(Tl[-1], T[-1])
        assert np.array_equal(b, basis)


def test_run_pivots_timed_graph_matches_untimed(eng_cls):
    """bench.py's timed region (one hipGraph with event nodes around every
    elimination) computes exactly what the plain pivot loop computes."""
    from simplex_amd import synth
    T, basis = synth.full_tableau("dense", 300, 500, 21)
    outs = []
    for kw in (dict(time_elim=True, use_graph=True), dict(time_elim=True, use_graph=False),
               dict(time_elim=False, use_graph=True)):
        with eng_cls(0) as e:
            e.set_ld_pad(64)
            e.load(T, basis)
            e.run_pivots(5)
            e.sync()
            e.elim_timing(reset=True)
            e.run_pivots(40, **kw)
            e.sync()
            ms, cnt, cols = e.elim_timing(reset=True)
            if kw["time_elim"]:
                assert cnt == 40 and ms > 0 and cols > 0
            outs.append((e.history().tolist(), e.tableau()))
    for h, t in outs[1:]:
        assert h == outs[0][0] and np.array_equal(t, outs[0][1])
    ref, rb = T.copy(), basis.copy()
    st, hist = O.solve_tableau(ref, rb, max_iters=45)
    assert [tuple(x) for x in outs[0][0]] == hist and np.array_equal(outs[0][1], ref)


@pytest.mark.parametrize("pad", [0, 2, 64, 130])
def test_ld_padding_is_transparent(eng_cls, pad):
    from simplex_amd import synth
    T, basis = synth.full_tableau("dense", 257, 300, 4)
    ref, rb = T.copy(), basis.copy()
    st, hist = O.solve_tableau(ref, rb)
    with eng_cls(0) as e:
        e.set_ld_pad(pad)
        e.load(T, basis)
        r = e.solve()
        assert [tuple(x) for x in e.history().tolist()] == hist
        assert np.array_equal(e.tableau(), ref) and r.objective == ref[-1, -1]


# ----------------------------------------------------------- linprog adapter, controller
LP_CASES = [
    dict(c=[-3, -5], A_ub=[[1, 0], [0, 2], [3, 2]], b_ub=[4, 12, 18]),
    dict(c=[50, 80], A_ub=[[-4, -1], [-1, -6], [-4, -6]], b_ub=[-4, -6, -12]),
    dict(c=[-1, -1], A_ub=[[1, 1], [-1, -1], [2, 1]], b_ub=[10, -10, 15], A_eq=[[1, 1]],
         b_eq=[10]),
    dict(c=[-1], A_ub=[[1], [-1]], b_ub=[5, -10]),                       # infeasible
    dict(c=[-1, -1], A_ub=[[1, -1]], b_ub=[1]),                           # unbounded
    dict(c=[1, -2, 3], A_ub=[[1, 1, 1], [1, -1, 0]], b_ub=[7, 2], A_eq=[[0, 1, 1]], b_eq=[3],
         bounds=[(-1, 4), (None, 5), (0, None)]),                          # shifted / free
]


@pytest.mark.parametrize("case", LP_CASES)
def test_linprog_adapter_vs_highs(case):
    from scipy.optimize import linprog as highs
    from simplex_amd.linprog import linprog as gpu
    kw = {k: v for k, v in case.items() if k != "c"}
    a = gpu(case["c"], method="highs-ds", options={"presolve": True, "time_limit": 10}, **kw)
    b = highs(case["c"], method="highs-ds", **kw)
    assert a.status == b.status and a.success == b.success
    if b.status == 0:
        assert abs(a.fun - b.fun) <= 1e-9 * max(1.0, abs(b.fun))


def test_linprog_adapter_random_dense_vs_highs():
    from scipy.optimize import linprog as highs
    from simplex_amd.linprog import linprog as gpu
    rng = np.random.default_rng(5)
    for k in range(6):
        m, n = 30 + 7 * k, 20 + 5 * k
        A = rng.uniform(-1, 2, size=(m, n))
        b = rng.uniform(1, 10, size=m)
        c = -rng.uniform(0, 1, size=n)
        a, h = gpu(c, A_ub=A, b_ub=b), highs(c, A_ub=A, b_ub=b, method="highs-ds")
        assert a.status == h.status
        if h.status == 0:
            assert abs(a.fun - h.fun) <= 1e-9 * max(1.0, abs(h.fun))


@pytest.mark.parametrize("engine", ["highs", "gpu"])
def test_controller_end_to_end_real_solvers(tmp_path, monkeypatch, engine):
    """reference tests/test_solver_controller.py MAX case, unmocked: the tables
    come from the GPU pivot engine, the answer from HiGHS or the GPU."""
    from simplex_amd import storage
    from simplex_amd.controller import SolverController
    monkeypatch.setattr(storage, "OUTPUT_DIR", str(tmp_path))
    wrap = {"problema_definicion": {
        "funcion_objetivo": {"type": "maximize", "coefficients": {"x1": 15.0, "x2": 18.0}},
        "restricciones": [
            {"coefficients": {"x1": 4.0, "x2": 2.0}, "operator": "<=", "rhs": 2000.0},
            {"coefficients": {"x1": 2.0, "x2": 6.0}, "operator": "<=", "rhs": 2400.0},
            {"coefficients": {"x1": 20.0, "x2": 28.0}, "operator": "<=", "rhs": 14000.0}]}}
    rep = SolverController(wrap, answer_engine=engine).run()
    sol = rep["solucion_encontrada"]
    assert sol["status"] == "Solucion Factible"
    assert sol["valor_optimo_z"] == pytest.approx(9833.333333333, rel=1e-9)
    tabs = rep["tablas_intermedias"]
    assert [t["pivot"] for t in tabs] == [None, (1, 1), (2, 0), (0, 3)]
    assert tabs[-1]["table"][-1][-1] == pytest.approx(9833.3333, abs=1e-4)
    assert "<table" in rep["visualizacion_gilp_html"]
    assert len(list(tmp_path.iterdir())) == 1


def test_config5_degenerate_bland_full_size_first_pivots(eng_cls):
    """BASELINE config 5 (m = n = 4096 degenerate LP, Bland): basis indices
    bit-exact after every one of the first pivots vs the oracle."""
    from simplex_amd import synth
    m = n = 4096
    T, basis = synth.full_tableau("degenerate", m, n, 5)
    ref, rb = T.copy(), basis.copy()
    seen = []
    st, hist = O.solve_tableau(ref, rb, rule="bland", max_iters=25,
                               on_pivot=lambda r, c, _T: seen.append(rb.copy()))
    with eng_cls(0) as e:
        e.load(T, basis)
        del T
        for k in range(len(hist)):
            assert e.pivot(rule="bland") == hist[k]
            assert np.array_equal(e.basis(), seen[k])
        assert np.array_equal(e.tableau(), ref)
        # keep going: Bland never cycles; the objective never decreases
        z0 = e.objective_row()[-1]
        r = e.solve(rule="bland", max_iters=400)
        assert r.status in (0, 1) and e.objective_row()[-1] >= z0


def test_sharded_rccl_in_timed_graph(eng_cls):
    """bench.py --gpus N path: RCCL all-gather / all-reduce captured in the
    event-timed hipGraph (1-rank communicator on the single test GPU)."""
    from simplex_amd import dist, synth
    m, n = 600, 900
    T, basis = synth.full_tableau("dense", m, n, 8)
    ref, rb = T.copy(), basis.copy()
    st, hist = O.solve_tableau(ref, rb, max_iters=70)
    uid = dist.make_unique_id()
    with dist.ShardedTableau(0, 0, 1, uid) as s:
        s.load_shard(T[:-1], T[-1], basis, m, 0)
        s.run_pivots(10, use_graph=True)
        s.sync()
        s.elim_timing(reset=True)
        s.run_pivots(60, time_elim=True, use_graph=True)
        s.sync()
        ms, cnt, cols = s.elim_timing(reset=True)
        assert cnt == 60 and ms > 0
        assert [tuple(h) for h in s.history().tolist()] == hist
        assert np.array_equal(s.tableau(), ref)


@pytest.mark.parametrize("window,k", [(0, 4), (24, 30)])
def test_config4_eight_virtual_ranks_full_size(eng_cls, window, k):
    """BASELINE config 4: the config-3 tableau (8192 x 16385) row-sharded over
    8 ranks (1024 rows each), here 8 virtual ranks on one GPU exchanging
    in-process; first pivots bit-exact vs the oracle on every rank.  window 24:
    the bench's N > 1 path (a full window and a partial one)."""
    from simplex_amd import dist, synth
    m = n = 8192
    world = 8
    uid = b"cfg4" + os.urandom(124)
    outs, errors = {}, []

    def rank_main(rank):
        try:
            r0, r1 = dist.row_partition(m, world, rank)
            Tl, obj, basis = synth.tableau_rows("dense", m, n, 20251205, r0, r1, order="F")
            with dist.ShardedTableau(0, rank, world, uid, local=True) as s:
                s.set_window(window)
                s.load_shard(Tl, obj, basis, m, r0)
                s.solve(max_iters=k)
                outs[rank] = (r0, r1, s.history().tolist(), s.tableau(), s.basis())
        except Exception as ex:  # pragma: no cover
            errors.append(ex)

    th = [threading.Thread(target=rank_main, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=900)
    assert not errors, errors
    T, basis = synth.full_tableau("dense", m, n, 20251205)
    st, hist = O.solve_tableau(T, basis, max_iters=k)
    for rank in range(world):
        r0, r1, h, Tl, b = outs[rank]
        assert [tuple(x) for x in h] == hist
        assert np.array_equal(Tl[:-1], T[r0:r1]) and np.array_equal(Tl[-1], T[-1])
        assert np.array_equal(b, basis)


def test_device_phase2_objective_and_row_gather_match_host(eng_cls):
    from simplex_amd import lp
    rng = np.random.default_rng(12)
    m, N = 37, 90
    T = rng.normal(size=(m + 1, N))
    T[rng.random(T.shape) < 0.2] = 0.0
    basis = rng.permutation(N - 1)[:m].astype(np.int64)
    cost = rng.normal(size=N - 1)
    cost[rng.random(N - 1) < 0.3] = 0.0
    with eng_cls(0) as e:
        e.load(T, basis)
        for i in (0, 5, m - 1):
            assert e.row(i).tobytes() == T[i].tobytes()
        e.set_phase2_objective(cost)
        got = e.objective_row()
    ref = lp.phase2_objective(T, basis, cost)
    assert got.tobytes() == ref.tobytes()
    assert np.array_equal(ref, O.phase2_row(T, basis, cost))
