"""Report persistence with the reference's ``StorageService`` API.

Mirrors ``app/services/storage_service.py`` (reference): sequential files
``outputs/<prefix><N>.json`` under the same prefixes (``app/config.py:20-24``),
the same save / load-latest entry points and the same return values
(``save_*`` -> path, ``load_*`` -> data, ``FileNotFoundError`` when nothing was
saved yet, ``None`` for an unreadable file).  The controller calls
``save_solution`` once per solve (``solver_controller.py:426``); the reference
tests patch that static method (``tests/test_solver_controller.py:126``).

What changes, for many concurrent ``/solve`` calls and large reports:

* **No check-then-write race.**  The reference picks the first number whose
  file does not exist (``storage_service.py:34-42``) and opens it later, so two
  concurrent solves can pick the same name and one report overwrites the other.
  Here a number is claimed by creating the file with ``O_CREAT | O_EXCL``; the
  content goes to a private temporary file that replaces the claimed name
  atomically, so a reader never sees a half-written report.
* **Latest = latest complete.**  ``load_*`` take the highest-numbered file that
  holds a complete document; a number that is claimed but still being written
  (an empty placeholder) is skipped instead of raising ``JSONDecodeError``.
* **Bounded writes.**  ``json.dump`` streams to the file (the report is never
  rendered as one string).  Long numeric tables (``tablas_intermedias`` rows,
  pivot histories) are written one row per line instead of one number per line
  as ``indent=4`` would (the byte count of a 2M-cell history drops ~3x), and the
  engine already caps snapshots at 2,000,000 cells.

Storage is a sink of the hot path, not part of it: nothing here touches the GPU.
"""
from __future__ import annotations

import json
import os
import re
import tempfile
from typing import Any, Dict, List, Optional

OUTPUT_DIR = os.environ.get("SPX_OUTPUT_DIR", os.path.join(os.getcwd(), "outputs"))
# the reference's prefixes (app/config.py:20-24)
PREFIX_FUNCION_OBJETIVO = "funcion_objetivo"
PREFIX_RESTRICCIONES = "restricciones"
PREFIX_SOLUCION = "solucion_"
PREFIX_PROBLEMA = "problema_"
PREFIX_PDF = "reporte_solucion_"
# kept for callers of the round-1 module
PREFIX_SOLUTION = PREFIX_SOLUCION


def _out_dir() -> str:
    return OUTPUT_DIR


class StorageService:
    """Sequential JSON files in OUTPUT_DIR (reference: storage_service.py:24-182)."""

    def __init__(self):
        # (the reference creates OUTPUT_DIR here; this build creates it on the
        # first save, so constructing a controller has no file-system effect)
        pass

    # --- file names -------------------------------------------------------

    @staticmethod
    def _claim_next_filename(prefix: str, extension: str = ".json") -> str:
        """Create and return the first free ``<prefix><N><extension>`` (O_EXCL:
        the name belongs to this caller even under concurrent claims)."""
        d = _out_dir()
        os.makedirs(d, exist_ok=True)
        number = 1
        while True:
            path = os.path.join(d, f"{prefix}{number}{extension}")
            try:
                fd = os.open(path, os.O_WRONLY | os.O_CREAT | os.O_EXCL, 0o644)
            except FileExistsError:
                number += 1
                continue
            os.close(fd)
            return path

    @staticmethod
    def _get_next_filename(prefix: str, extension: str = ".json") -> str:
        """The reference's name picker (storage_service.py:34-42), race-free: the
        returned name is claimed (an empty file exists under it)."""
        return StorageService._claim_next_filename(prefix, extension)

    @staticmethod
    def _numbered(prefix: str, extension: str) -> List[tuple]:
        d = _out_dir()
        if not os.path.exists(d):
            return []
        pat = re.compile(f"^{re.escape(prefix)}(\\d+){re.escape(extension)}$")
        out = []
        for f in os.listdir(d):
            m = pat.match(f)
            if m:
                out.append((int(m.group(1)), os.path.join(d, f)))
        out.sort()
        return out

    @staticmethod
    def _get_latest_filename(prefix: str, extension: str = ".json") -> Optional[str]:
        """Highest-numbered ``<prefix><N><extension>`` that is not an empty
        placeholder (storage_service.py:44-72), or None."""
        for _, path in reversed(StorageService._numbered(prefix, extension)):
            try:
                if os.path.getsize(path) > 0:
                    return path
            except OSError:
                continue
        return None

    # --- save -------------------------------------------------------------

    @staticmethod
    def save_json(data: Any, prefix: str, extension: str = ".json") -> Optional[str]:
        """Write ``data`` to a new sequential file; the path, or None on an I/O
        error (the reference prints the error and returns None, :76-88)."""
        filename = None
        try:
            # the claim creates OUTPUT_DIR and the name: an unwritable directory
            # is an I/O error like any other (None, as the reference returns)
            filename = StorageService._claim_next_filename(prefix, extension)
            _write_atomic(filename, data)
            return filename
        except (IOError, OSError) as e:
            print(f"Error al guardar el archivo {filename or prefix}: {e}")
            return None

    @staticmethod
    def save_constraints(constraints: List[Dict]) -> Optional[str]:
        return StorageService.save_json(constraints, prefix=PREFIX_RESTRICCIONES)

    @staticmethod
    def save_objective_function(objective_data: Dict) -> Optional[str]:
        return StorageService.save_json(objective_data, prefix=PREFIX_FUNCION_OBJETIVO)

    @staticmethod
    def save_solution(report_data: Dict) -> Optional[str]:
        return StorageService.save_json(report_data, prefix=PREFIX_SOLUCION)

    @staticmethod
    def save_problem(problem_data: dict) -> Optional[str]:
        return StorageService.save_json(problem_data, prefix=PREFIX_PROBLEMA)

    # --- load -------------------------------------------------------------

    @staticmethod
    def load_json(prefix: str) -> Any:
        """Data of the latest complete ``<prefix><N>.json`` (storage_service.py:
        124-144): FileNotFoundError if none, None if it cannot be parsed."""
        filename = StorageService._get_latest_filename(prefix, extension=".json")
        if not filename or not os.path.exists(filename):
            raise FileNotFoundError(
                f"No se encontró ningún archivo con prefijo '{prefix}' en {_out_dir()}.")
        try:
            with open(filename, "r", encoding="utf-8") as f:
                return json.load(f)
        except json.JSONDecodeError:
            print(f"Error: El archivo {filename} está corrupto o mal formateado.")
            return None
        except IOError as e:
            print(f"Error al leer el archivo {filename}: {e}")
            return None

    @staticmethod
    def load_constraints() -> List[Dict]:
        return StorageService.load_json(prefix=PREFIX_RESTRICCIONES)

    @staticmethod
    def load_objective_function() -> Dict:
        return StorageService.load_json(prefix=PREFIX_FUNCION_OBJETIVO)

    @staticmethod
    def load_problem() -> dict:
        return StorageService.load_json(prefix=PREFIX_PROBLEMA)

    @staticmethod
    def load_solution() -> dict:
        return StorageService.load_json(prefix=PREFIX_SOLUCION)

    @staticmethod
    def get_new_pdf_path() -> str:
        """A claimed path for the next PDF report (storage_service.py:176-179)."""
        return StorageService._claim_next_filename(prefix=PREFIX_PDF, extension=".pdf")


# --- writing --------------------------------------------------------------

def _read_umask() -> int:
    """The process umask without changing it: /proc/self/status ('Umask:'),
    else the os.umask round trip -- done once, at import, before any /solve
    thread runs (os.umask(0) would briefly open files created meanwhile by
    other threads to 0666)."""
    try:
        with open("/proc/self/status") as f:
            for line in f:
                if line.startswith("Umask:"):
                    return int(line.split()[1], 8)
    except (OSError, ValueError, IndexError):
        pass
    m = os.umask(0o022)
    os.umask(m)
    return m


_UMASK = _read_umask()


def _process_umask() -> int:
    return _UMASK


def _write_atomic(path: str, data: Any) -> None:
    """Stream ``data`` as JSON to a temporary file beside ``path``, then move it
    over ``path`` (a reader sees the empty claim or the whole document)."""
    d = os.path.dirname(path) or "."
    fd, tmp = tempfile.mkstemp(prefix=".tmp_", suffix=".json", dir=d)
    try:
        # mkstemp creates 0600; the report keeps the mode a plain open() gives
        # (0666 & ~umask), as the reference's json.dump target has
        os.fchmod(fd, 0o666 & ~_process_umask())
        with os.fdopen(fd, "w", encoding="utf-8") as f:
            _dump(data, f, 0)
            f.write("\n")
        os.replace(tmp, path)
    except BaseException:
        try:
            os.unlink(tmp)
        except OSError:
            pass
        raise


_IND = "    "  # the reference's indent=4


def _scalar(x) -> bool:
    return x is None or isinstance(x, (bool, int, float, str))


_enc_str = json.encoder.encode_basestring  # (the C encoder where CPython has it)


def _scalar_dict_body(o: dict, level: int) -> Optional[str]:
    """The lines of a dict whose values are all non-string scalars, exactly as
    the generic branch of ``_dump`` writes them, built with C-level loops: the
    keys through the string encoder, the values through ONE ``json.dumps`` of
    the value list split on its ", " separators (a number, true / false / null
    never contains one).  A constraint's coefficient dict of config 2 has
    2,048 entries and a report holds 1,024 of them: one write per entry was
    ~5 s of save_solution (profiles/r06/user_path.json).  None: not such a
    dict (the generic branch runs)."""
    vals = list(o.values())
    if not all(_scalar(v) and not isinstance(v, str) for v in vals):
        return None
    enc = json.dumps(vals, ensure_ascii=False, allow_nan=True)[1:-1].split(", ")
    ind = _IND * (level + 1)
    keys = [ind + _enc_str(str(k)) + ": " for k in o]
    return ",\n".join(map(str.__add__, keys, enc))


def _dump(o: Any, f, level: int) -> None:
    """``json.dump(o, indent=4, ensure_ascii=False)`` except that a list of
    scalars (a table row, a pivot pair) goes on one line, streamed piecewise."""
    o = _jsonable(o) if not isinstance(o, (dict, list, str, int, float, bool, type(None))) else o
    if isinstance(o, dict):
        if not o:
            f.write("{}")
            return
        body = _scalar_dict_body(o, level) if len(o) > 8 else None
        if body is not None:
            f.write("{\n" + body + "\n" + _IND * level + "}")
            return
        f.write("{\n")
        n = len(o)
        for k, (key, val) in enumerate(o.items()):
            f.write(_IND * (level + 1) + json.dumps(str(key), ensure_ascii=False) + ": ")
            _dump(val, f, level + 1)
            f.write(",\n" if k + 1 < n else "\n")
        f.write(_IND * level + "}")
    elif isinstance(o, list):
        if not o:
            f.write("[]")
            return
        if all(_scalar(x) for x in o):
            f.write(json.dumps(o, ensure_ascii=False, allow_nan=True))
            return
        f.write("[\n")
        n = len(o)
        for k, val in enumerate(o):
            f.write(_IND * (level + 1))
            _dump(val, f, level + 1)
            f.write(",\n" if k + 1 < n else "\n")
        f.write(_IND * level + "]")
    else:
        f.write(json.dumps(o, ensure_ascii=False, allow_nan=True))


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
