"""ctypes binding of oracle/build/libspx_oracle.so — TEST INFRASTRUCTURE ONLY
(tests/ checker and bench.py cpu_baseline; never imported by the product)."""
from __future__ import annotations

import ctypes
import os

import numpy as np

_SO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "build", "libspx_oracle.so")
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            raise FileNotFoundError(f"{_SO} missing: run `make -C oracle`")
        _lib = ctypes.CDLL(_SO)
        i64, dp, lp = ctypes.c_int64, ctypes.POINTER(ctypes.c_double), \
            ctypes.POINTER(ctypes.c_int64)
        _lib.spxo_solve.argtypes = [dp, i64, i64, lp, ctypes.c_int, ctypes.c_double,
                                    ctypes.c_double, i64, i64, ctypes.c_int, lp, i64, lp]
        _lib.spxo_solve.restype = ctypes.c_int
        _lib.spxo_pivot.argtypes = [dp, i64, i64, i64, i64, ctypes.c_int]
        _lib.spxo_threads.restype = ctypes.c_int
        _lib.spxo_set_threads.argtypes = [ctypes.c_int]
        _lib.spxo_set_threads.restype = ctypes.c_int
    return _lib


def threads() -> int:
    return lib().spxo_threads()


def set_threads(n: int) -> int:
    """OpenMP threads for the following calls (n <= 0 keeps the count); returns it."""
    return lib().spxo_set_threads(int(n))


def solve(T: np.ndarray, basis: np.ndarray, rule="dantzig", eps_opt=1e-9, eps_piv=1e-12,
          n_enter=0, max_iters=0, skip_zero=True, hist_cap=1 << 20):
    """In place on a C-contiguous float64 T and int64 basis; returns (status, hist)."""
    assert T.flags.c_contiguous and T.dtype == np.float64
    assert basis.flags.c_contiguous and basis.dtype == np.int64
    hist = np.zeros(2 * hist_cap, dtype=np.int64)
    n = ctypes.c_int64()
    st = lib().spxo_solve(T.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), T.shape[0],
                          T.shape[1], basis.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                          1 if rule == "bland" else 0, eps_opt, eps_piv, n_enter, max_iters,
                          1 if skip_zero else 0,
                          hist.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), hist_cap,
                          ctypes.byref(n))
    k = min(n.value, hist_cap)
    return st, [(int(hist[2 * i]), int(hist[2 * i + 1])) for i in range(k)]
