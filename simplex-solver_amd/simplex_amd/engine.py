"""Device-resident simplex tableau: the Python face of libspx.so.

``DeviceTableau`` owns one spx context (one HIP stream + the tableau in HBM).
It is what ``simplex_amd.simple_simplex.optimize_json_format`` (the drop-in
for the reference's ``simple_simplex`` pivot engine, called at
app/controllers/solver_controller.py:318) pivots on.

Tableau convention: ``T`` has m+1 rows, objective row LAST in
the "z_j - c_j" form of a MAX problem, right-hand side in the last column;
``basis[i]`` is the variable basic in row i.
"""
from __future__ import annotations

import atexit
import ctypes
import os
import threading
from dataclasses import dataclass

import numpy as np

from . import _lib as L

RULES = {"dantzig": L.SPX_RULE_DANTZIG, "bland": L.SPX_RULE_BLAND}
STATUS_NAMES = {L.SPX_OPTIMAL: "optimal", L.SPX_ITER_LIMIT: "iteration_limit",
                L.SPX_INFEASIBLE: "infeasible", L.SPX_UNBOUNDED: "unbounded",
                L.SPX_RUNNING: "running"}


class SpxError(RuntimeError):
    """A libspx call failed (HIP / RCCL / argument error)."""


@dataclass
class SolveResult:
    status: int          # scipy OptimizeResult.status numbering (0,1,2,3)
    iters: int
    objective: float     # objective-row RHS (MAX form)
    elapsed_s: float

    @property
    def status_name(self) -> str:
        return STATUS_NAMES.get(self.status, str(self.status))


def _dptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


def _lptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_int64))


def make_opts(rule="dantzig", eps_opt=1e-9, eps_piv=1e-12, max_iters=0, time_limit=0.0,
              n_enter=0, chunk=32, use_graph=True, skip_zero_cols=True) -> L.SpxOpts:
    if isinstance(rule, str):
        if rule.lower() not in RULES:
            raise ValueError(f"unknown pivot rule {rule!r}; expected one of {sorted(RULES)}")
        rule = RULES[rule.lower()]
    o = L.default_opts()
    o.rule = int(rule)
    o.eps_opt = float(eps_opt)
    o.eps_piv = float(eps_piv)
    o.max_iters = int(max_iters or 0)
    o.time_limit_s = float(time_limit or 0.0)
    o.n_enter = int(n_enter or 0)
    o.chunk = int(chunk)
    o.use_graph = 1 if use_graph else 0
    o.skip_zero_cols = 1 if skip_zero_cols else 0
    return o


def auto_window(m: int, cols: int) -> int:
    """Window size (pivots per tableau pass) for a solve to
    optimality on an m x cols constraint block: none for small tableaux (the
    single-pivot path is launch-bound there either way), 8 from ~1M cells,
    16 from ~8M, 24 from ~64M (profiles/r01/bench_configs.jsonl, bench K sweep)."""
    cells = int(m) * int(cols)
    if cells < (1 << 20):
        return 0
    if cells < (1 << 23):
        return 8
    if cells < (1 << 26):
        return 16
    return 24


class DeviceTableau:
    """A tableau resident on one GPU (or one row shard of it, see dist.py)."""

    def __init__(self, device: int = 0, *, _sharded=None):
        self._lib = L.lib()
        self._ctx = ctypes.c_void_p()
        self.sharded = _sharded is not None
        if _sharded is None:
            rc = self._lib.spx_create(ctypes.byref(self._ctx), int(device))
        else:
            rank, nranks, uid, local = _sharded
            if local == "peer":  # no communicator: the persistent chain's peers only
                rc = self._lib.spx_create_sharded_peer(ctypes.byref(self._ctx), int(device),
                                                       int(rank), int(nranks))
            else:
                create = (self._lib.spx_create_sharded_local if local
                          else self._lib.spx_create_sharded)
                rc = create(ctypes.byref(self._ctx), int(device), int(rank), int(nranks), uid)
        if rc != 0:
            msg = self._err()
            self.close()
            raise SpxError(f"spx_create failed ({rc}): {msg}")
        self.device = device
        self.m = self.m_local = self.N = self.row0 = 0

    # -- plumbing -----------------------------------------------------------
    def _err(self) -> str:
        if not self._ctx:
            return "no context"
        s = self._lib.spx_last_error(self._ctx)
        return s.decode() if s else ""

    def _check(self, rc: int, what: str) -> int:
        if rc < 0:
            raise SpxError(f"{what} failed ({rc}): {self._err()}")
        return rc

    def close(self) -> None:
        if getattr(self, "_ctx", None):
            self._lib.spx_destroy(self._ctx)
            self._ctx = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):  # pragma: no cover - best effort
        try:
            self.close()
        except Exception:
            pass

    def _refresh_dims(self):
        mg, ml, n, r0 = (ctypes.c_int64() for _ in range(4))
        self._lib.spx_dims(self._ctx, ctypes.byref(mg), ctypes.byref(ml), ctypes.byref(n),
                           ctypes.byref(r0))
        self.m, self.m_local, self.N, self.row0 = mg.value, ml.value, n.value, r0.value

    # -- data in ------------------------------------------------------------
    def load(self, T, basis) -> "DeviceTableau":
        """Load a full (m+1) x N tableau (objective row last) and its basis."""
        T = np.asarray(T, dtype=np.float64)
        if T.ndim != 2 or T.shape[0] < 1 or T.shape[1] < 1:
            raise ValueError("tableau must be a non-empty 2-D array")
        m = T.shape[0] - 1
        basis = np.ascontiguousarray(np.asarray(basis, dtype=np.int64).reshape(-1))
        if basis.shape[0] != m:
            raise ValueError(f"basis has {basis.shape[0]} entries, tableau has {m} rows")
        if np.isfortran(T) and not T.flags.c_contiguous:
            layout, ld = L.SPX_COL_MAJOR, T.shape[0]
        else:
            T = np.ascontiguousarray(T)
            layout, ld = L.SPX_ROW_MAJOR, T.shape[1]
        self._check(self._lib.spx_load(self._ctx, _dptr(T), T.shape[0], T.shape[1], ld, layout,
                                       _lptr(basis)), "spx_load")
        self._refresh_dims()
        return self

    def load_rows(self, A, obj, basis, m_global: int, row0: int) -> "DeviceTableau":
        """Load constraint rows [row0, row0 + A.shape[0]) plus the objective row."""
        A = np.asarray(A, dtype=np.float64)
        if A.ndim != 2:
            raise ValueError("A must be 2-D")
        obj = np.ascontiguousarray(np.asarray(obj, dtype=np.float64).reshape(-1))
        basis = np.ascontiguousarray(np.asarray(basis, dtype=np.int64).reshape(-1))
        if obj.shape[0] != A.shape[1]:
            raise ValueError("objective row length != number of columns")
        if basis.shape[0] != m_global:
            raise ValueError("basis length != m_global")
        if np.isfortran(A) and not A.flags.c_contiguous:
            layout, ld = L.SPX_COL_MAJOR, max(1, A.shape[0])
        else:
            A = np.ascontiguousarray(A)
            layout, ld = L.SPX_ROW_MAJOR, A.shape[1]
        self._check(self._lib.spx_load_rows(self._ctx, _dptr(A), A.shape[0], A.shape[1], ld,
                                            layout, _dptr(obj), _lptr(basis), int(m_global),
                                            int(row0)), "spx_load_rows")
        self._refresh_dims()
        return self

    def set_objective(self, obj) -> None:
        obj = np.ascontiguousarray(np.asarray(obj, dtype=np.float64).reshape(-1))
        if obj.shape[0] != self.N:
            raise ValueError("objective row length != number of columns")
        self._check(self._lib.spx_set_objective(self._ctx, _dptr(obj)), "spx_set_objective")

    # -- data out -----------------------------------------------------------
    def tableau(self) -> np.ndarray:
        out = np.empty((self.m_local + 1, self.N), dtype=np.float64)
        self._check(self._lib.spx_get_tableau(self._ctx, _dptr(out), self.N, L.SPX_ROW_MAJOR),
                    "spx_get_tableau")
        return out

    def objective_row(self) -> np.ndarray:
        out = np.empty(self.N, dtype=np.float64)
        self._check(self._lib.spx_get_objective(self._ctx, _dptr(out)), "spx_get_objective")
        return out

    def basis(self) -> np.ndarray:
        out = np.empty(max(self.m, 0), dtype=np.int64)
        if self.m:
            self._check(self._lib.spx_get_basis(self._ctx, _lptr(out)), "spx_get_basis")
        return out

    def column(self, j: int) -> np.ndarray:
        out = np.empty(self.m_local, dtype=np.float64)
        self._check(self._lib.spx_get_column(self._ctx, int(j), _dptr(out)), "spx_get_column")
        return out

    def row(self, i: int) -> np.ndarray:
        out = np.empty(self.N, dtype=np.float64)
        self._check(self._lib.spx_get_row(self._ctx, int(i), _dptr(out)), "spx_get_row")
        return out

    def set_phase2_objective(self, cost) -> None:
        """obj = -cost + sum_i cost[basis[i]] * T[i,:] on the device (row order)."""
        cost = np.ascontiguousarray(np.asarray(cost, dtype=np.float64).reshape(-1))
        if cost.shape[0] != self.N - 1:
            raise ValueError("cost must have N-1 entries")
        self._check(self._lib.spx_set_phase2_objective(self._ctx, _dptr(cost)),
                    "spx_set_phase2_objective")

    def history(self) -> np.ndarray:
        """(k, 2) int64 array of (row, col) pivots since load."""
        n = ctypes.c_int64()
        self._check(self._lib.spx_get_history(self._ctx, None, 0, ctypes.byref(n)),
                    "spx_get_history")
        k = n.value
        out = np.empty((k, 2), dtype=np.int64)
        if k:
            self._check(self._lib.spx_get_history(self._ctx, _lptr(out), k, ctypes.byref(n)),
                        "spx_get_history")
        return out

    # -- pivoting -----------------------------------------------------------
    def solve(self, **kw) -> SolveResult:
        o = make_opts(**kw)
        res = L.SpxResult()
        rc = self._lib.spx_solve(self._ctx, ctypes.byref(o), ctypes.byref(res))
        self._check(rc, "spx_solve")
        return SolveResult(int(res.status), int(res.iters), float(res.objective),
                           float(res.elapsed_s))

    def pivot(self, **kw):
        """One rule-chosen pivot: returns (r, c), or the terminal status
        (L.SPX_OPTIMAL / L.SPX_UNBOUNDED) when no pivot is possible."""
        o = make_opts(**kw)
        r, c = ctypes.c_int64(), ctypes.c_int64()
        rc = self._check(self._lib.spx_pivot(self._ctx, ctypes.byref(o), ctypes.byref(r),
                                             ctypes.byref(c)), "spx_pivot")
        if rc == L.SPX_RUNNING:
            return int(r.value), int(c.value)
        return rc

    def pivot_at(self, r: int, c: int) -> None:
        self._check(self._lib.spx_pivot_at(self._ctx, int(r), int(c)), "spx_pivot_at")

    def run_pivots(self, npivots: int, time_elim: int = 0, **kw) -> None:
        """Enqueue npivots pivots; time_elim = k > 0 brackets every k-th
        elimination with HIP events (read them with elim_timing)."""
        o = make_opts(**kw)
        self._check(self._lib.spx_run_pivots(self._ctx, ctypes.byref(o), int(npivots),
                                             int(time_elim)), "spx_run_pivots")

    def sync(self) -> None:
        self._check(self._lib.spx_sync(self._ctx), "spx_sync")

    def state(self):
        st, it, z = ctypes.c_int32(), ctypes.c_int64(), ctypes.c_double()
        self._check(self._lib.spx_state(self._ctx, ctypes.byref(st), ctypes.byref(it),
                                        ctypes.byref(z)), "spx_state")
        return int(st.value), int(it.value), float(z.value)

    def elim_timing(self, reset: bool = True):
        """(total_ms, launches, touched_columns) of event-timed eliminations."""
        ms, cnt, cols = ctypes.c_double(), ctypes.c_int64(), ctypes.c_int64()
        self._check(self._lib.spx_elim_timing(self._ctx, ctypes.byref(ms), ctypes.byref(cnt),
                                              ctypes.byref(cols), 1 if reset else 0),
                    "spx_elim_timing")
        return float(ms.value), int(cnt.value), int(cols.value)

    def elim_variant(self) -> dict:
        """The elimination / flush configuration in use.  Keys: R, row_chunks,
        col_groups, nt_flags, interleave, pipeline (bit 0 software pipelining,
        bit 1 XCD swizzle), ld, and for the window flush: flush_var, flush_map,
        flush_row_chunks, flush_groups (the last two from the last flush launch)."""
        out = np.zeros(7, dtype=np.int64)
        self._check(self._lib.spx_get_elim_variant(self._ctx, _lptr(out)),
                    "spx_get_elim_variant")
        keys = ("R", "row_chunks", "col_groups", "nt_flags", "interleave", "pipeline", "ld")
        d = {k: int(v) for k, v in zip(keys, out)}
        fo = np.zeros(4, dtype=np.int64)
        self._check(self._lib.spx_get_flush_variant(self._ctx, _lptr(fo)),
                    "spx_get_flush_variant")
        d.update(flush_var=int(fo[0]), flush_map=int(fo[1]), flush_row_chunks=int(fo[2]),
                 flush_groups=int(fo[3]))
        return d

    def set_window(self, K: int) -> None:
        """Windowed elimination: K pivots per pass over the tableau (0/1 = off)."""
        self._check(self._lib.spx_set_window(self._ctx, int(K)), "spx_set_window")


    def set_row_fix_fold(self, on: bool = True) -> None:
        """The row_fix fold (spx_set_row_fix_fold): a window's
        leaving rows are rewritten inside the next window's chain launch (on)
        or by a row_fix launch after every window (off, the default: the fold
        measured no faster)."""
        self._check(self._lib.spx_set_row_fix_fold(self._ctx, 1 if on else 0),
                    "spx_set_row_fix_fold")
    def set_chain(self, mode: int = 0, min_blocks: int = 0) -> None:
        """Pivot chain of a window: 0 = one persistent launch per window when
        the tableau fits (default), 1 = two launches per pivot (lazy kernels),
        2 / 3 = persistent with 256- / 512-thread blocks.
        Bit-identical either way; min_blocks raises the persistent grid."""
        self._check(self._lib.spx_set_chain(self._ctx, int(mode), int(min_blocks)),
                    "spx_set_chain")

    def set_chain_timing(self, on: bool = True) -> None:
        """HIP events around every window's pivot chain (diagnostic)."""
        self._check(self._lib.spx_set_chain_timing(self._ctx, 1 if on else 0),
                    "spx_set_chain_timing")

    def chain_timing(self, reset: bool = True):
        """(total_ms, windows) of the event-timed pivot chains."""
        ms, cnt = ctypes.c_double(), ctypes.c_int64()
        self._check(self._lib.spx_chain_timing(self._ctx, ctypes.byref(ms), ctypes.byref(cnt),
                                               1 if reset else 0), "spx_chain_timing")
        return float(ms.value), int(cnt.value)

    def chain_blocks(self) -> int:
        """Blocks of the persistent chain for the loaded tableau (0: not used)."""
        b = ctypes.c_int()
        self._check(self._lib.spx_get_chain(self._ctx, ctypes.byref(b)), "spx_get_chain")
        return int(b.value)

    def chain_stats(self) -> dict:
        """Admission record: calls run with the persistent chain, calls refused
        (launch-per-phase chain instead), blocks held now (spx_get_chain_stats)."""
        out = np.zeros(3, dtype=np.int64)
        self._check(self._lib.spx_get_chain_stats(self._ctx, _lptr(out)), "spx_get_chain_stats")
        return {"persistent_calls": int(out[0]), "refused_calls": int(out[1]),
                "blocks_held": int(out[2])}

    def set_chain_handshake(self, us: int = 0) -> None:
        """Start-handshake bound of persistent chains in us (0: automatic,
        20 us on one GPU / 100 ms for row shards; -k < 0: every k-th window
        (by epoch) aborts and is rerun, -1 every window -- test hooks).
        spx_set_chain_handshake."""
        self._check(self._lib.spx_set_chain_handshake(self._ctx, int(us)),
                    "spx_set_chain_handshake")

    def chain_reruns(self) -> int:
        """Windows rerun after their persistent chain found its blocks not
        co-resident (spx_get_chain_reruns)."""
        n = ctypes.c_int64()
        self._check(self._lib.spx_get_chain_reruns(self._ctx, ctypes.byref(n)),
                    "spx_get_chain_reruns")
        return int(n.value)

    @staticmethod
    def set_chain_budget(device: int, blocks: int) -> None:
        """Process-wide budget of persistent-chain blocks in flight on `device`
        (-1: default = the CU count or SPX_CHAIN_BUDGET; 0: never persistent)."""
        rc = L.lib().spx_set_chain_budget(int(device), int(blocks))
        if rc < 0:
            raise SpxError(f"spx_set_chain_budget failed ({rc})")

    def set_ld_pad(self, pad: int) -> None:
        """Extra doubles per stored column, applied at the next load."""
        self._check(self._lib.spx_set_ld_pad(self._ctx, int(pad)), "spx_set_ld_pad")

    def set_elim_variant(self, R: int = 0, target_wgs: int = 0, nt_flags: int = -1,
                         interleave: int = None, *, pipeline: bool = None, xcd: bool = None,
                         flush_variant: int = None, flush_map: int = None) -> None:
        """Elimination / flush tuning (spx_set_elim_variant, include/spx.h).

        R: rows per thread (2/4/8, 0 auto); target_wgs: grid target (0 auto);
        nt_flags: non-temporal bit 0 loads, bit 1 stores (-1 auto).  The C
        `interleave` word packs: bit 0 interleaved columns, bit 1 pipelining
        OFF, bit 2 XCD-aware swizzle, bits 8-10 window flush variant (only 0,
        the LDS-DMA ring, remains; others raise), bits 11-12 flush block map
        (bit 11 chunk-major, bit 12 groups rotated by row chunk; bit 13, the
        removed dynamic-claim flush, raises).  Pass `interleave` to set the whole word,
        or leave it None and give only the keyword fields to change: the others
        keep their current values (read back with elim_variant())."""
        if interleave is None:
            v = self.elim_variant()
            pipe = bool(v["pipeline"] & 1) if pipeline is None else bool(pipeline)
            xc = bool(v["pipeline"] & 2) if xcd is None else bool(xcd)
            fv = v["flush_var"] if flush_variant is None else int(flush_variant)
            fm = v["flush_map"] if flush_map is None else int(flush_map)
            interleave = (v["interleave"] & 1) | (0 if pipe else 2) | (4 if xc else 0)
            interleave |= (fv & 7) << 8 | (fm & 7) << 11
        self._check(self._lib.spx_set_elim_variant(self._ctx, int(R), int(target_wgs),
                                                   int(nt_flags), int(interleave)),
                    "spx_set_elim_variant")


class ContextPool:
    """Idle single-GPU contexts, reused by the solves of small LPs.

    The reference's user path (/solve, app/controllers/solver_controller.py:
    53-120, 290-319) solves textbook-sized LPs, where creating and destroying
    an spx context (a HIP stream, events, pinned host State, device buffers:
    ~2 ms each way, tests/test_gpu_user_path.py) costs more than the pivots.
    ``lp.solve_standard_form`` therefore takes a context from this pool and
    gives it back: at most `cap` idle contexts per device (SPX_CONTEXT_POOL,
    default 8; 0 disables), only for tableaux of at most `max_cells` cells (a
    pooled context keeps its last tableau in HBM), never one whose solve
    raised.  Thread-safe (the reference's /solve runs from many threads,
    tests/test_performance_load.py:80-83); a forked child never reuses its
    parent's contexts (a HIP context does not survive fork)."""

    def __init__(self, cap: int | None = None, max_cells: int = 1 << 22):
        self.cap = int(os.environ.get("SPX_CONTEXT_POOL", "8")) if cap is None else cap
        self.max_cells = max_cells
        self._lock = threading.Lock()
        self._idle: dict = {}
        self._pid = os.getpid()

    def _fresh(self) -> None:
        if self._pid != os.getpid():  # (held by the lock's owner)
            self._idle = {}
            self._pid = os.getpid()

    def acquire(self, device: int = 0) -> "DeviceTableau":
        with self._lock:
            self._fresh()
            free = self._idle.get(device)
            eng = free.pop() if free else None
        if eng is None:
            return DeviceTableau(device)
        eng.set_window(0)  # (the knob lp.py's solves change; the load resets the rest)
        return eng

    def release(self, eng: "DeviceTableau", reusable: bool = True) -> None:
        keep = (reusable and self.cap > 0 and not eng.sharded and getattr(eng, "_ctx", None)
                and (eng.m_local + 1) * eng.N <= self.max_cells)
        if keep:
            with self._lock:
                self._fresh()
                free = self._idle.setdefault(eng.device, [])
                if len(free) < self.cap:
                    free.append(eng)
                    return
        eng.close()

    def clear(self) -> None:
        with self._lock:
            idle, self._idle = self._idle, {}
            mine = self._pid == os.getpid()
        if mine:
            for free in idle.values():
                for eng in free:
                    eng.close()


POOL = ContextPool()
atexit.register(POOL.clear)

