"""ctypes binding of libspx.so (the C-ABI declared in include/spx.h).

This is the only place Python touches the native engine.  There is no CPU
fallback: if the library (or the HIP runtime it links) cannot be loaded, every
engine call raises ``SpxLibraryError`` loudly.
"""
from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SPX_LIB", os.path.join(_HERE, "lib", "libspx.so"))

# status / return codes (include/spx.h)
SPX_OK = 0
SPX_OPTIMAL = 0
SPX_ITER_LIMIT = 1
SPX_INFEASIBLE = 2
SPX_UNBOUNDED = 3
SPX_RUNNING = 4
SPX_E_ARG = -1
SPX_E_HIP = -2
SPX_E_RCCL = -3
SPX_E_STATE = -4
SPX_E_NOPEER = -6

SPX_RULE_DANTZIG = 0
SPX_RULE_BLAND = 1
SPX_ROW_MAJOR = 0
SPX_COL_MAJOR = 1


class SpxLibraryError(RuntimeError):
    """libspx.so is missing or could not be loaded (no silent fallback)."""


class SpxOpts(ctypes.Structure):
    _fields_ = [
        ("rule", ctypes.c_int32),
        ("skip_zero_cols", ctypes.c_int32),
        ("eps_opt", ctypes.c_double),
        ("eps_piv", ctypes.c_double),
        ("max_iters", ctypes.c_int64),
        ("time_limit_s", ctypes.c_double),
        ("n_enter", ctypes.c_int64),
        ("chunk", ctypes.c_int32),
        ("use_graph", ctypes.c_int32),
    ]


class SpxResult(ctypes.Structure):
    _fields_ = [
        ("status", ctypes.c_int32),
        ("pad", ctypes.c_int32),
        ("iters", ctypes.c_int64),
        ("objective", ctypes.c_double),
        ("elapsed_s", ctypes.c_double),
    ]


_P = ctypes.c_void_p
_I64 = ctypes.c_int64
_I32 = ctypes.c_int32
_DP = ctypes.POINTER(ctypes.c_double)
_LP = ctypes.POINTER(ctypes.c_int64)

# name -> (restype, argtypes); every entry point of include/spx.h
SIGNATURES = {
    "spx_default_opts": (None, [ctypes.POINTER(SpxOpts)]),
    "spx_abi_version": (ctypes.c_int, []),
    "spx_create": (ctypes.c_int, [ctypes.POINTER(_P), ctypes.c_int]),
    "spx_destroy": (ctypes.c_int, [_P]),
    "spx_last_error": (ctypes.c_char_p, [_P]),
    "spx_comm_unique_id": (ctypes.c_int, [ctypes.c_char_p]),
    "spx_create_sharded": (ctypes.c_int, [ctypes.POINTER(_P), ctypes.c_int, ctypes.c_int,
                                          ctypes.c_int, ctypes.c_char_p]),
    "spx_create_sharded_local": (ctypes.c_int, [ctypes.POINTER(_P), ctypes.c_int, ctypes.c_int,
                                                ctypes.c_int, ctypes.c_char_p]),
    "spx_load": (ctypes.c_int, [_P, _DP, _I64, _I64, _I64, ctypes.c_int, _LP]),
    "spx_load_rows": (ctypes.c_int, [_P, _DP, _I64, _I64, _I64, ctypes.c_int, _DP, _LP, _I64,
                                     _I64]),
    "spx_set_objective": (ctypes.c_int, [_P, _DP]),
    "spx_get_tableau": (ctypes.c_int, [_P, _DP, _I64, ctypes.c_int]),
    "spx_get_objective": (ctypes.c_int, [_P, _DP]),
    "spx_get_basis": (ctypes.c_int, [_P, _LP]),
    "spx_get_column": (ctypes.c_int, [_P, _I64, _DP]),
    "spx_get_row": (ctypes.c_int, [_P, _I64, _DP]),
    "spx_set_phase2_objective": (ctypes.c_int, [_P, _DP]),
    "spx_get_history": (ctypes.c_int, [_P, _LP, _I64, _LP]),
    "spx_dims": (ctypes.c_int, [_P, _LP, _LP, _LP, _LP]),
    "spx_solve": (ctypes.c_int, [_P, ctypes.POINTER(SpxOpts), ctypes.POINTER(SpxResult)]),
    "spx_pivot": (ctypes.c_int, [_P, ctypes.POINTER(SpxOpts), _LP, _LP]),
    "spx_pivot_at": (ctypes.c_int, [_P, _I64, _I64]),
    "spx_run_pivots": (ctypes.c_int, [_P, ctypes.POINTER(SpxOpts), _I64, ctypes.c_int]),
    "spx_sync": (ctypes.c_int, [_P]),
    "spx_state": (ctypes.c_int, [_P, ctypes.POINTER(_I32), _LP, _DP]),
    "spx_elim_timing": (ctypes.c_int, [_P, _DP, _LP, _LP, ctypes.c_int]),
    "spx_set_ld_pad": (ctypes.c_int, [_P, ctypes.c_int]),
    "spx_set_window": (ctypes.c_int, [_P, ctypes.c_int]),
    "spx_set_row_fix_fold": (ctypes.c_int, [_P, ctypes.c_int]),
    "spx_set_chain": (ctypes.c_int, [_P, ctypes.c_int, ctypes.c_int]),
    "spx_set_chain_timing": (ctypes.c_int, [_P, ctypes.c_int]),
    "spx_chain_timing": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_double),
                                        ctypes.POINTER(ctypes.c_int64), ctypes.c_int]),
    "spx_get_chain": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_int)]),
    "spx_set_chain_budget": (ctypes.c_int, [ctypes.c_int, ctypes.c_int]),
    "spx_create_sharded_peer": (ctypes.c_int, [ctypes.POINTER(_P), ctypes.c_int, ctypes.c_int,
                                               ctypes.c_int]),
    "spx_peer_blob_size": (ctypes.c_int, []),
    "spx_peer_export": (ctypes.c_int, [_P, ctypes.c_void_p, _I64]),
    "spx_peer_import": (ctypes.c_int, [_P, ctypes.c_char_p, ctypes.c_int]),
    "spx_peer_chain_local": (ctypes.c_int, [_P]),
    "spx_set_peer_push": (ctypes.c_int, [_P, ctypes.c_int]),
    "spx_get_peer_push": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_int)]),
    "spx_peer_debug": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]),
    "spx_peer_pool_debug": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]),
    "spx_peer_groups": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int),
                                       ctypes.POINTER(ctypes.c_int)]),
    "spx_get_chain_stats": (ctypes.c_int, [_P, _LP]),
    "spx_set_chain_handshake": (ctypes.c_int, [_P, _I64]),
    "spx_chain_shm_path": (ctypes.c_int, [ctypes.c_int, ctypes.c_char_p, ctypes.c_int]),
    "spx_get_chain_reruns": (ctypes.c_int, [_P, _LP]),
    "spx_get_elim_variant": (ctypes.c_int, [_P, _LP]),
    "spx_get_flush_variant": (ctypes.c_int, [_P, _LP]),
    "spx_set_elim_variant": (ctypes.c_int, [_P, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                            ctypes.c_int]),
}

_lib = None
_lock = threading.Lock()


def lib() -> ctypes.CDLL:
    """Load libspx.so once (thread-safe) and return it; raise loudly if absent."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise SpxLibraryError(
                f"libspx.so not found at {LIB_PATH}; build it with "
                "`python -c 'import __graft_entry__ as g; g.build()'` (hipcc, gfx950)")
        try:
            handle = ctypes.CDLL(LIB_PATH)
        except OSError as e:  # pragma: no cover - environment dependent
            raise SpxLibraryError(f"cannot load {LIB_PATH}: {e}") from e
        # SPX_LIB_PARTIAL=1: tolerate symbols an older build lacks (same-box
        # A/B of two library builds only; the product binds everything)
        partial = os.environ.get("SPX_LIB_PARTIAL") == "1"
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(handle, name, None)
            if fn is None:
                if partial:
                    continue
                raise SpxLibraryError(f"{LIB_PATH} lacks {name}")
            fn.restype = res
            fn.argtypes = args
        if handle.spx_abi_version() != 1:
            raise SpxLibraryError("libspx ABI version mismatch")
        _lib = handle
        return _lib


def default_opts() -> SpxOpts:
    o = SpxOpts()
    lib().spx_default_opts(ctypes.byref(o))
    return o
