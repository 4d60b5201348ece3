"""Minimal report sink with the reference's ``StorageService.save_solution`` seam.

The reference persists the report as sequential ``outputs/solucion_N.json``
files (app/services/storage_service.py:34-42, :75-88, :106-112).  Storage is out
of scope for this build; this keeps only the static ``save_solution`` entry the
controller calls once per solve (solver_controller.py:426) and that the
reference tests patch (tests/test_solver_controller.py:126).  File names are
claimed with O_EXCL, so concurrent solves cannot overwrite each other (the
reference's _get_next_filename has a check-then-write race).
"""
from __future__ import annotations

import json
import os

OUTPUT_DIR = os.environ.get("SPX_OUTPUT_DIR", os.path.join(os.getcwd(), "outputs"))
PREFIX_SOLUTION = "solucion_"


class StorageService:
    @staticmethod
    def save_solution(report: dict) -> str:
        os.makedirs(OUTPUT_DIR, exist_ok=True)
        k = 1
        while True:
            path = os.path.join(OUTPUT_DIR, f"{PREFIX_SOLUTION}{k}.json")
            try:
                fd = os.open(path, os.O_WRONLY | os.O_CREAT | os.O_EXCL, 0o644)
            except FileExistsError:
                k += 1
                continue
            with os.fdopen(fd, "w", encoding="utf-8") as f:
                json.dump(report, f, ensure_ascii=False, indent=2, default=_jsonable)
            return path


def _jsonable(o):
    try:
        import numpy as np
        if isinstance(o, np.ndarray):
            return o.tolist()
        if isinstance(o, np.generic):
            return o.item()
    except ImportError:  # pragma: no cover
        pass
    if isinstance(o, tuple):
        return list(o)
    raise TypeError(f"not JSON serialisable: {type(o).__name__}")
