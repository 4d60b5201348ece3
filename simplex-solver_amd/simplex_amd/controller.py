"""``SolverController`` with the reference's API surface, pivoting on the GPU.

Mirrors app/controllers/solver_controller.py so the Flask ``/solve`` route
(ui_controller.py:194-195) and the reference tests see the same object:
  * ``SolverController(problem_data_wrapper)`` (:33-50) — variables sorted
    lexicographically (:46);
  * ``run() -> dict | None`` (:53-120) — None when the objective or the
    constraints are missing (:65-67) or on any exception (:112-120);
  * the answer comes from the module-level ``linprog`` (:76-85, the tests'
    mock seam), the per-pivot tables from the pivot engine (:290-363), now
    ``simplex_amd.simple_simplex`` backed by libspx.so (HIP, gfx950);
  * the report dict (:417-422) and the single ``StorageService.save_solution``
    call (:426), with the same console lines the tests assert on.
The reference's "Plan A" (gilp plotly HTML, :207-255) is out of scope: the
visualisation HTML is the static tableau HTML of its Plan B (:190-200).
"""
from __future__ import annotations

import os
import traceback
from typing import Any, Dict, List, Tuple

import numpy as np
from scipy.optimize import linprog  # answer path + mock seam (:9, :78-85)

from .linprog import linprog as gpu_linprog
from .storage import StorageService
from .simple_simplex import (add_constraint, add_objective, create_tableau,
                             optimize_json_format)

SOLVER_OPTIONS = {"presolve": True, "time_limit": 10}  # :76
OP_CODE = {"<=": "L", ">=": "G", "=": "E"}             # :306
PIVOT_STYLE = 'style="background-color:#fff0f0; color:#d00; font-weight:bold;"'
TABLE_OPEN = ('<table class="table table-bordered table-striped" style="border:1px solid '
              '#ccc; justify-content:center; float:none; margin-left:auto; margin-right:auto;">')


class SolverController:
    def __init__(self, problem_data_wrapper: dict, answer_engine: str | None = None):
        """answer_engine: "highs" (default, the reference's scipy/HiGHS call
        through the module-level ``linprog`` seam) or "gpu" (simplex_amd.linprog,
        the same two-phase GPU engine that produces the tables)."""
        self.answer_engine = (answer_engine or os.environ.get("SPX_ANSWER_ENGINE", "highs")).lower()
        if self.answer_engine not in ("highs", "gpu"):
            raise ValueError(f"unknown answer engine {self.answer_engine!r}")
        self.storage = StorageService()
        definition = (problem_data_wrapper or {}).get("problema_definicion", {})
        self.objective_data = definition.get("funcion_objetivo")
        self.constraints_data = definition.get("restricciones")
        coeffs = (self.objective_data or {}).get("coefficients", {}) if self.objective_data else {}
        self.variables = sorted(coeffs.keys())
        print("SolverController inicializado con datos en memoria.")

    # ------------------------------------------------------------------ run
    def run(self):
        print("=== 3. Solución del Problema ===")
        if self.objective_data is None or self.constraints_data is None:
            print("Error: El solver no recibió datos válidos en la inicialización.")
            return None
        try:
            print("Preparando modelo para el solver (Scipy)...")
            c, A_ub, b_ub, A_eq, b_eq, bounds = self._prepare_model_for_scipy(
                self.objective_data, self.constraints_data, self.variables)
            print("Ejecutando solver principal (Scipy)...")
            solve = linprog if self.answer_engine == "highs" else gpu_linprog
            result = solve(c, A_ub=A_ub, b_ub=b_ub, A_eq=A_eq, b_eq=b_eq, bounds=bounds,
                           method="highs-ds", options=dict(SOLVER_OPTIONS))
            if result.success:
                print("Generando visualización (tablas del motor de pivoteo)...")
                html, tables = self._generate_visualization_html_and_tables()
            else:
                print("Problema infactible o no acotado. Omitiendo visualización.")
                html = "<p>Visualización no disponible (Problema infactible o no acotado).</p>"
                tables = []
            return self._display_and_save_results(result, self.objective_data["type"], html,
                                                  tables)
        except KeyError as e:
            print(f"Error inesperado: No se encontró la llave {e} en los archivos JSON.")
            print("Parece que los archivos JSON no tienen el formato esperado.")
            return None
        except Exception as e:  # noqa: BLE001 - reference behaviour (:116-120)
            print(f"Ha ocurrido un error inesperado durante el cálculo: {e}")
            traceback.print_exc()
            return None

    # ------------------------------------------------------- model for linprog
    def _prepare_model_for_scipy(self, objective_data: dict, constraints_data: list,
                                 variables: list):
        coefficients = objective_data["coefficients"]
        c = [coefficients.get(v, 0) for v in variables]
        if objective_data["type"] == "maximize":  # linprog minimises (:133-134)
            c = [-x for x in c]
        A_ub, b_ub, A_eq, b_eq = [], [], [], []
        for const in constraints_data:
            row = [const["coefficients"].get(v, 0) for v in variables]
            op, rhs = const["operator"], const["rhs"]
            if op == "<=":
                A_ub.append(row)
                b_ub.append(rhs)
            elif op == ">=":
                A_ub.append([-x for x in row])
                b_ub.append(-rhs)
            elif op == "=":
                # the reference keeps the row in A_eq AND as two A_ub rows (:154-161)
                A_eq.append(row)
                b_eq.append(rhs)
                A_ub.append(row)
                b_ub.append(rhs)
                A_ub.append([-x for x in row])
                b_ub.append(-rhs)
        bounds = [(0, None) for _ in variables]
        as_np = lambda v: np.array(v) if v else None  # noqa: E731
        return np.array(c), as_np(A_ub), as_np(b_ub), as_np(A_eq), as_np(b_eq), bounds

    # ------------------------------------------------------- pivot engine
    def _run_simple_simplex(self) -> dict:
        tab = create_tableau(number_of_variables=len(self.variables),
                             number_of_constraints=len(self.constraints_data))
        for const in self.constraints_data:
            coeffs = ",".join(str(const["coefficients"].get(v, 0)) for v in self.variables)
            op = OP_CODE.get(const["operator"], "E")
            add_constraint(tab, f"{coeffs},{op},{const['rhs']}")
        is_max = self.objective_data["type"] == "maximize"
        obj = ",".join(str(self.objective_data["coefficients"].get(v, 0))
                       for v in self.variables)
        add_objective(tab, f"{obj},{'1' if is_max else '0'}")
        return optimize_json_format(tab, maximize=is_max)

    def _extract_tableaus_from_simple_simplex(self, simplex_json: dict) -> List[Dict[str, Any]]:
        out: List[Dict[str, Any]] = []
        for step in simplex_json.get("pivotSteps", []) if simplex_json else []:
            num = step.get("step", "?")
            r, c = step.get("pivotRowIndex"), step.get("pivotColIndex")
            data = step.get("tableau", [])
            if not data:
                continue
            headers = ["Base"] + [f"C{i}" for i in range(len(data[0]))]
            if num == 0 or r is None:
                title = "Iteración 0 (Tabla Inicial)"
            else:
                title = f"Iteración {num} (Pivote: Fila {r}, Col {c})"
            table = [headers]
            for i, row in enumerate(data):
                table.append([f"F{i}"] + [round(v, 4) if isinstance(v, (int, float)) else v
                                          for v in row])
            out.append({"iteration": num, "title": title, "table": table,
                        "pivot": (r, c) if r is not None and c is not None else None})
        return out

    def _tableau_to_html(self, tableau_list: list, pivot_r, pivot_c) -> str:
        pr = -1 if pivot_r is None else pivot_r
        pc = -1 if pivot_c is None else pivot_c
        parts = [TABLE_OPEN]
        for ri, row in enumerate(tableau_list):
            parts.append("<tr>")
            for ci, cell in enumerate(row):
                tag = "th" if ci == 0 or ri == 0 else "td"
                style = PIVOT_STYLE if (ri == pr + 1 and ci == pc + 1) else ""
                text = f"{cell:.4f}" if isinstance(cell, float) else cell
                parts.append(f"<{tag} {style}>{text}</{tag}>")
            parts.append("</tr>")
        parts.append("</table>")
        return "".join(parts)

    def _generate_visualization_html_and_tables(self) -> Tuple[str, List[Dict[str, Any]]]:
        print("Ejecutando motor de pivoteo (GPU) para extraer tablas...")
        try:
            tables = self._extract_tableaus_from_simple_simplex(self._run_simple_simplex())
            html = "<br>".join(
                f"<h4>{t.get('title', 'Tabla')}</h4>" + self._tableau_to_html(
                    t.get("table", []), *(t["pivot"] if t.get("pivot") else (None, None)))
                for t in tables)
            print("Motor de pivoteo completado exitosamente.")
            return html, tables
        except Exception as e:  # noqa: BLE001 - Plan B errors become HTML (:203-205)
            print(f"Error crítico en Plan B (simple_simplex): {e}")
            return f"<p>Error en Plan B: {e}</p>", []

    # ------------------------------------------------------- report
    def _display_and_save_results(self, result, objective_type: str, html: str, tables: list):
        print("----------------------------------")
        print("         SOLUCIÓN ÓPTIMA          ")
        print("----------------------------------")
        definition = {"funcion_objetivo": self.objective_data,
                      "restricciones": self.constraints_data}
        if result.success:
            print("¡Se encontró una solución factible! \n")
            print("Valores de las variables:")
            values = {}
            for i, name in enumerate(self.variables):
                values[name] = result.x[i]
                print(f"   {name} = {result.x[i]:.4f}")
            print("\nValor de la Función Objetivo (Z):")
            z = -result.fun if objective_type == "maximize" else result.fun
            print(f"   Z = {z:.4f}")
            found = {"status": "Solucion Factible", "mensaje_solver": result.message,
                     "valores_variables": values, "valor_optimo_z": z}
        else:
            status = "Sin Solucion Factible" if result.status == 2 else "Error"
            print(f"{status} ")
            if result.status != 2:
                print(f"(Estado: {result.message})")
            found = {"status": status, "mensaje_solver": result.message,
                     "valores_variables": None, "valor_optimo_z": None}
        report = {"problema_definicion": definition, "solucion_encontrada": found,
                  "visualizacion_gilp_html": html, "tablas_intermedias": tables}
        try:
            filename = StorageService.save_solution(report)
            print(f"\nReporte de solución guardado en: {filename}")
        except Exception as e:  # noqa: BLE001
            print(f"\nAdvertencia: No se pudo guardar el reporte de solución: {e}")
        return report
