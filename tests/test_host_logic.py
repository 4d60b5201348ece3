"""Host-side logic that needs no GPU: standard form, generators, the
simple_simplex text API, the SolverController contract (reference
tests/test_solver_controller.py re-expressed with unittest.mock)."""
import io
import os
from contextlib import redirect_stdout
from unittest import mock

import numpy as np
import pytest
from scipy.optimize import OptimizeResult

from oracle import simplex_oracle as O
from simplex_amd import lp, simple_simplex as ss, synth
from simplex_amd.controller import SolverController

CASES = [
    ([3, 5], [([1, 0], "<=", 4), ([0, 2], "<=", 12), ([3, 2], "<=", 18)], True),
    ([50, 80], [([4, 1], ">=", 4), ([1, 6], ">=", 6), ([4, 6], ">=", 12)], False),
    ([1, 1], [([1, 1], "=", 10), ([2, 1], "<=", 15)], True),
    ([1, 1], [([-1, -2], "<=", -4), ([3, 1], "<=", 9)], False),
    ([1, 1], [], True),
]


@pytest.mark.parametrize("c,rows,mx", CASES)
def test_standard_form_matches_oracle(c, rows, mx):
    sf = lp.build_standard_form(c, rows, mx)
    o = O.standard_form(c, rows, mx)
    assert np.array_equal(sf.T, o["T"]) and np.array_equal(sf.basis, o["basis"])
    assert (sf.n, sf.m, sf.k) == (o["n"], o["m"], o["k"])
    assert np.array_equal(sf.cost, o["cost"])


def test_phase2_objective_matches_oracle():
    rng = np.random.default_rng(0)
    T = rng.normal(size=(6, 11))
    basis = np.array([0, 3, 5, 2, 9], dtype=np.int64)
    cost = rng.normal(size=10)
    assert np.array_equal(lp.phase2_objective(T, basis, cost), O.phase2_row(T, basis, cost))


@pytest.mark.parametrize("kind", ["dense", "degenerate"])
def test_synth_row_blocks_are_rank_independent(kind):
    m, n = 37, 23
    full, basis = synth.full_tableau(kind, m, n, seed=4)
    parts = []
    for r0, r1 in [(0, 10), (10, 11), (11, 37)]:
        T, obj, b = synth.tableau_rows(kind, m, n, 4, r0, r1, order="F")
        assert np.array_equal(obj, full[-1]) and np.array_equal(b, basis)
        parts.append(np.asarray(T))
    assert np.array_equal(np.vstack(parts), full[:-1])


def test_dense_generator_is_feasible_and_positive():
    A, b, c = synth.dense_lp(50, 40, 1)
    assert A.min() >= 0.1 and A.max() < 1.0 and b.min() >= 10 and c.min() >= 0.1


def test_simple_simplex_text_api_parsing():
    t = ss.create_tableau(number_of_variables=2, number_of_constraints=2)
    ss.add_constraint(t, "1.0,2.0,L,4.0")
    ss.add_constraint(t, "3,1,G,2")
    ss.add_objective(t, "3.0,5.0,1")
    assert t.rows == [([1.0, 2.0], "L", 4.0), ([3.0, 1.0], "G", 2.0)]
    assert t.c == [3.0, 5.0] and t.maximize_flag is True
    with pytest.raises(ValueError):
        ss.add_constraint(t, "1,2,L,3")  # too many constraints
    t2 = ss.create_tableau(2, 1)
    with pytest.raises(ValueError):
        ss.add_constraint(t2, "1,2,X,3")
    with pytest.raises(ValueError):
        ss.add_constraint(t2, "1,L,3")
    with pytest.raises(ValueError):
        ss.add_objective(t2, "1,2,7")
    with pytest.raises(ValueError):
        ss.optimize_json_format(t2, maximize=True)  # objective missing


# --- SolverController contract (reference tests/test_solver_controller.py) ----
MAX_OBJ = {"type": "maximize", "coefficients": {"x1": 15.0, "x2": 18.0}}
MAX_CONS = [{"coefficients": {"x1": 4.0, "x2": 2.0}, "operator": "<=", "rhs": 2000.0},
            {"coefficients": {"x1": 2.0, "x2": 6.0}, "operator": "<=", "rhs": 2400.0},
            {"coefficients": {"x1": 20.0, "x2": 28.0}, "operator": "<=", "rhs": 14000.0}]
MIN_OBJ = {"type": "minimize", "coefficients": {"x1": 50.0, "x2": 80.0}}
MIN_CONS = [{"coefficients": {"x1": 4.0, "x2": 1.0}, "operator": ">=", "rhs": 4.0},
            {"coefficients": {"x1": 1.0, "x2": 6.0}, "operator": ">=", "rhs": 6.0},
            {"coefficients": {"x1": 4.0, "x2": 6.0}, "operator": ">=", "rhs": 12.0}]
MAX_RES = OptimizeResult({"fun": -9833.333333333334, "success": True, "status": 0,
                          "x": np.array([388.8888888888889, 222.22222222222223]),
                          "message": "Optimization successful."})


def _wrap(obj, cons):
    return {"problema_definicion": {"funcion_objetivo": obj, "restricciones": cons}}


def test_prepare_model_maximize():
    ctl = SolverController(_wrap(MAX_OBJ, MAX_CONS))
    c, A_ub, b_ub, A_eq, b_eq, bounds = ctl._prepare_model_for_scipy(MAX_OBJ, MAX_CONS,
                                                                     ctl.variables)
    assert np.array_equal(c, [-15.0, -18.0])
    assert np.array_equal(A_ub, [[4, 2], [2, 6], [20, 28]])
    assert A_eq is None and bounds == [(0, None), (0, None)]


def test_prepare_model_minimize_and_equality():
    ctl = SolverController(_wrap(MIN_OBJ, MIN_CONS))
    c, A_ub, *_ = ctl._prepare_model_for_scipy(MIN_OBJ, MIN_CONS, ctl.variables)
    assert np.array_equal(c, [50.0, 80.0])
    assert np.array_equal(A_ub, [[-4, -1], [-1, -6], [-4, -6]])
    eq = [{"coefficients": {"x1": 1.0, "x2": 1.0}, "operator": "=", "rhs": 10.0}]
    _, A_ub, b_ub, A_eq, b_eq, _ = ctl._prepare_model_for_scipy(MIN_OBJ, eq, ["x1", "x2"])
    assert np.array_equal(A_eq, [[1, 1]]) and np.array_equal(b_eq, [10])
    assert np.array_equal(A_ub, [[1, 1], [-1, -1]]) and np.array_equal(b_ub, [10, -10])


def test_variables_sorted_lexicographically():
    obj = {"type": "maximize", "coefficients": {"x2": 1, "x10": 1, "x1": 1}}
    assert SolverController(_wrap(obj, []) ).variables == ["x1", "x10", "x2"]


def test_run_maximize_contract_with_mocks():
    with mock.patch("simplex_amd.controller.linprog", return_value=MAX_RES), \
         mock.patch("simplex_amd.controller.StorageService.save_solution",
                    return_value="outputs/solucion_mock.json") as save, \
         mock.patch("simplex_amd.controller.SolverController._run_simple_simplex",
                    side_effect=RuntimeError("no GPU in this container")):
        buf = io.StringIO()
        with redirect_stdout(buf):
            rep = SolverController(_wrap(MAX_OBJ, MAX_CONS)).run()
    out = buf.getvalue()
    assert "¡Se encontró una solución factible!" in out
    assert "x1 = 388.8889" in out and "x2 = 222.2222" in out and "Z = 9833.3333" in out
    assert "Reporte de solución guardado en: outputs/solucion_mock.json" in out
    save.assert_called_once()
    for r in (rep, save.call_args[0][0]):
        assert r["solucion_encontrada"]["status"] == "Solucion Factible"
        assert r["solucion_encontrada"]["valor_optimo_z"] == pytest.approx(9833.333333)
        assert r["problema_definicion"]["funcion_objetivo"] == MAX_OBJ
    # Plan B failure is reported as HTML, tables empty (solver_controller.py:203-205)
    assert "Error en Plan B" in rep["visualizacion_gilp_html"]
    assert rep["tablas_intermedias"] == []


def test_run_infeasible_and_missing_data():
    fail = OptimizeResult({"success": False, "status": 2, "message": "Infeasible."})
    with mock.patch("simplex_amd.controller.linprog", return_value=fail), \
         mock.patch("simplex_amd.controller.StorageService.save_solution",
                    return_value="x.json") as save:
        buf = io.StringIO()
        with redirect_stdout(buf):
            rep = SolverController(_wrap(MAX_OBJ, MAX_CONS)).run()
        assert "Sin Solucion Factible " in buf.getvalue()
        assert rep["solucion_encontrada"]["valor_optimo_z"] is None
        save.assert_called_once()
    with mock.patch("simplex_amd.controller.StorageService.save_solution") as save:
        buf = io.StringIO()
        with redirect_stdout(buf):
            assert SolverController(problem_data_wrapper={}).run() is None
        assert "Error: El solver no recibió datos válidos en la inicialización." in \
            buf.getvalue()
        save.assert_not_called()


def test_extract_tables_and_html():
    ctl = SolverController(_wrap(MAX_OBJ, MAX_CONS))
    js = {"pivotSteps": [
        {"step": 0, "pivotRowIndex": None, "pivotColIndex": None, "tableau": [[1.0, 2.0]]},
        {"step": 1, "pivotRowIndex": 0, "pivotColIndex": 1, "tableau": [[0.123456, 1.0]]},
        {"step": 2, "pivotRowIndex": 0, "pivotColIndex": 0, "tableau": []}]}
    tabs = ctl._extract_tableaus_from_simple_simplex(js)
    assert [t["title"] for t in tabs] == ["Iteración 0 (Tabla Inicial)",
                                         "Iteración 1 (Pivote: Fila 0, Col 1)"]
    assert tabs[1]["table"] == [["Base", "C0", "C1"], ["F0", 0.1235, 1.0]]
    html = ctl._tableau_to_html(tabs[1]["table"], 0, 1)
    assert "<td style=" in html and "1.0000" in html


def test_storage_service_writes_unique_files(tmp_path, monkeypatch):
    from simplex_amd import storage
    monkeypatch.setattr(storage, "OUTPUT_DIR", str(tmp_path))
    a = storage.StorageService.save_solution({"a": np.float64(1.5), "t": (1, 2)})
    b = storage.StorageService.save_solution({"b": 2})
    assert a != b and a.endswith("solucion_1.json") and b.endswith("solucion_2.json")


def test_auto_window_by_size():
    """The two-phase driver's window choice: off for small
    tableaux, growing with the cell count; always a size spx_set_window takes."""
    from simplex_amd.engine import auto_window
    assert auto_window(3, 7) == 0
    assert auto_window(1024, 3073) == 8          # config 2
    assert auto_window(4096, 8193) == 16         # config 5
    assert auto_window(8192, 16385) == 24        # config 3
    for m, n in ((0, 0), (10, 10), (2000, 600), (5000, 20000), (100000, 200000)):
        assert auto_window(m, n) in (0, 8, 16, 24)


# --- report persistence (simplex_amd/storage.py) ---------------

def test_storage_roundtrip_and_latest(tmp_path, monkeypatch):
    """save_* / load_* mirror app/services/storage_service.py: sequential names
    per prefix, load_* returns the highest-numbered complete document."""
    import json
    from simplex_amd import storage
    S = storage.StorageService
    monkeypatch.setattr(storage, "OUTPUT_DIR", str(tmp_path))
    with pytest.raises(FileNotFoundError):
        S.load_solution()
    rep = {"problema_definicion": {"funcion_objetivo": {"type": "maximize"}},
           "tablas_intermedias": [{"iteration": 0, "table": [["F0", 1.0, np.float64(2.5)],
                                                           ["F1", -0.0, float("nan")]],
                                   "pivot": (1, 2)}],
           "valor": np.float32(3.0), "arr": np.arange(3)}
    p1 = S.save_solution(rep)
    p2 = S.save_solution({"n": 2})
    assert p1.endswith("solucion_1.json") and p2.endswith("solucion_2.json")
    assert S.load_solution() == {"n": 2}
    back = json.load(open(p1, encoding="utf-8"))
    t = back["tablas_intermedias"][0]
    assert t["pivot"] == [1, 2] and t["table"][0] == ["F0", 1.0, 2.5]
    assert back["valor"] == 3.0 and back["arr"] == [0, 1, 2]
    assert np.isnan(t["table"][1][2]) and str(t["table"][1][1]) == "-0.0"
    # a table row is one line (indent=4 would put every number on its own line)
    assert '["F0", 1.0, 2.5]' in open(p1, encoding="utf-8").read()
    for save, load in ((S.save_problem, S.load_problem), (S.save_constraints, S.load_constraints),
                       (S.save_objective_function, S.load_objective_function)):
        save({"k": [1, 2]})
        assert load() == {"k": [1, 2]}
    assert S.get_new_pdf_path().endswith("reporte_solucion_1.pdf")
    assert S.get_new_pdf_path().endswith("reporte_solucion_2.pdf")


def test_storage_scalar_dict_fast_path_same_bytes(monkeypatch):
    """The scalar-dict fast path of the report writer (a constraint's
    coefficient dict) gives the bytes the per-entry path gives, and both equal
    json.dumps(indent=4) for such a dict."""
    import io
    import json
    from simplex_amd import storage
    rng = np.random.default_rng(7)
    coef = {f"x{j:04d}": float(v) for j, v in enumerate(rng.standard_normal(300))}
    coef.update({"nan": float("nan"), "inf": float("inf"), "-inf": float("-inf"),
                 "negzero": -0.0, "int": 7, "big": 10 ** 30, "t": True, "f": False,
                 "none": None, 'q"uo\\te': 1.5, "línea\n\tñ": 2.0, "f64": np.float64(0.1)})
    doc = {"problema_definicion": {"funcion_objetivo": {"type": "maximize",
                                                        "coefficients": coef},
                                   "restricciones": [{"coefficients": coef, "operator": "<=",
                                                      "rhs": 4.0}] * 3},
           "valores": {f"x{j}": j * 0.5 for j in range(12)},
           "mixed": {f"k{j}": ("s" if j == 5 else j) for j in range(12)},
           "small": {"a": 1.0}}

    def dump():
        buf = io.StringIO()
        storage._dump(doc, buf, 0)
        return buf.getvalue()

    fast = dump()
    monkeypatch.setattr(storage, "_scalar_dict_body", lambda o, level: None)
    assert fast == dump()
    assert storage._scalar_dict_body.__name__ == "<lambda>"
    monkeypatch.undo()
    body = storage._scalar_dict_body(coef, 0)
    assert "{\n" + body + "\n}" == json.dumps(coef, indent=4, ensure_ascii=False)


def test_storage_latest_skips_claimed_placeholder(tmp_path, monkeypatch):
    """A number claimed by a solve still writing (empty file) is not 'latest'."""
    from simplex_amd import storage
    S = storage.StorageService
    monkeypatch.setattr(storage, "OUTPUT_DIR", str(tmp_path))
    S.save_solution({"v": 1})
    claimed = S._get_next_filename(storage.PREFIX_SOLUCION)
    assert claimed.endswith("solucion_2.json") and (tmp_path / "solucion_2.json").exists()
    assert S.load_solution() == {"v": 1}
    assert S.save_solution({"v": 3}).endswith("solucion_3.json")
    assert S.load_solution() == {"v": 3}
    (tmp_path / "solucion_4.json").write_text("{ not json")
    assert S.load_solution() is None   # the reference prints and returns None


def test_storage_concurrent_saves_unique_and_complete(tmp_path, monkeypatch):
    """Many threads saving at once (the reference's _get_next_filename can hand
    two of them one name): every report lands in its own complete file."""
    import json
    import threading
    from simplex_amd import storage
    S = storage.StorageService
    monkeypatch.setattr(storage, "OUTPUT_DIR", str(tmp_path))
    paths, errs = [], []

    def work(k):
        try:
            paths.append(S.save_solution({"k": k, "rows": [[k] * 50] * 20}))
        except Exception as e:  # pragma: no cover
            errs.append(e)

    th = [threading.Thread(target=work, args=(k,)) for k in range(32)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errs and len(set(paths)) == 32
    ks = sorted(json.load(open(p, encoding="utf-8"))["k"] for p in paths)
    assert ks == list(range(32))
    assert not [f for f in os.listdir(tmp_path) if f.startswith(".tmp_")]


def test_storage_report_mode_and_unwritable_dir(tmp_path, monkeypatch):
    """Saved reports keep the mode a plain open() gives (0666 & ~umask), and an
    unusable OUTPUT_DIR makes save_json return None instead of raising
    (reference storage_service.py:76-88 prints the error and returns None)."""
    import os
    import stat
    from simplex_amd import storage
    monkeypatch.setattr(storage, "OUTPUT_DIR", str(tmp_path))
    old = os.umask(0o022)
    try:
        path = storage.StorageService.save_solution({"a": 1})
    finally:
        os.umask(old)
    assert stat.S_IMODE(os.stat(path).st_mode) == 0o644
    blocker = tmp_path / "not_a_dir"
    blocker.write_text("x")
    monkeypatch.setattr(storage, "OUTPUT_DIR", str(blocker / "sub"))
    assert storage.StorageService.save_solution({"a": 1}) is None


def test_bench_all_cores_projection_bounds():
    """bench.py's all-physical-cores CPU figure (not measured: the harness
    gives the job 16 threads): linear scaling of the 16-thread rate, the
    last doubling's gain carried on, both capped by the host's DRAM roofline
    for the bytes one pivot moves."""
    import bench
    host = {"physical_cores": 128, "model": "AMD EPYC 9575F 64-Core Processor", "sockets": 2}
    bpp = bench.alg_bytes_per_pivot(8192, 8192)
    assert bpp == 16.0 * 8192 * 8193
    curve = {"1": 20.0, "2": 39.0, "4": 75.0, "8": 130.0, "16": 205.0}
    a = bench._all_cores_projection(205.0, 16, host, bpp, curve)
    roof = 2 * 614.4e9 / bpp
    assert a["measured"] is False and a["measured_scaling"] == curve
    assert abs(a["linear_projection"] - 205.0 * 8) < 1e-9
    assert abs(a["dram_roofline_pivots_per_s"] - roof) < 1e-6
    assert a["upper_bound"] == min(a["linear_projection"], roof)
    # three more doublings at 205/130 each, under the roofline here
    assert abs(a["doubling_extrapolation"] - min(205.0 * (205.0 / 130.0) ** 3, roof)) < 1e-6
    # unknown host model: no roofline, the linear figure bounds it
    b = bench._all_cores_projection(205.0, 16, dict(host, model="other"), bpp, curve)
    assert b["dram_roofline_pivots_per_s"] is None and b["upper_bound"] == 205.0 * 8


def test_row_transport_choice_is_deterministic_and_guarded():
    """bench.py's N > 1 transport trial: every rank passes the same
    all-reduced times, so every rank takes the same transport; push only when
    its self-test passed and it was faster (ties stay on pull)."""
    from simplex_amd.dist import choose_row_transport
    assert choose_row_transport(10.0, 8.0) == "push"
    assert choose_row_transport(8.0, 10.0) == "pull"
    assert choose_row_transport(8.0, 8.0) == "pull"
    assert choose_row_transport(10.0, 8.0, push_ok=False) == "pull"
    assert choose_row_transport(10.0, None) == "pull"
