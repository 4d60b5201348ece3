"""Row-sharded pivot protocol, restated on the CPU — TEST INFRASTRUCTURE ONLY.

Restates the exchange that libspx performs per pivot on a row-sharded
tableau (simplex-solver_amd/csrc/spx_capi.hip enqueue_pivot)
with torch.distributed collectives, so the protocol can be checked on CPU
(gloo, world size >= 2) against the single-process oracle:

  1. entering column: chosen locally from the replicated objective row;
  2. each rank packs [its best (ratio, tie, global row) key | that row
     normalised by its pivot-column entry] (prep_kernel);
  3. ONE all-gather of the packs; every rank takes the lexicographic winner
     (RCCL has no MINLOC) and the winner's row as p (norm_kernel<FINISH>);
  4. elimination of the local rows + the replicated objective row.
sharded_windowed_solve restates the windowed variant (the bench's N > 1
path, spx_delayed.hpp lazy_prep_kernel / lazy_norm_kernel<K, FINISH>): stale
local rows, the pivot column and the candidate row rebuilt from the pending
slots, the same single all-gather per pivot, one flush per K pivots.
The reference has no distributed code; the single-process
semantics it must reproduce are those of simplex_oracle.py.
"""
from __future__ import annotations

import numpy as np

from .simplex_oracle import BLAND, OPTIMAL, UNBOUNDED, ITER_LIMIT, select_entering

INF_KEY = (np.inf, np.iinfo(np.int64).max, -1)


def local_key(T_loc, row0, c, basis, rule, eps_piv):
    col = T_loc[:, c]
    best = INF_KEY
    for i in np.flatnonzero(col > eps_piv):
        ratio = T_loc[i, -1] / col[i]
        if np.isnan(ratio):
            continue
        g = row0 + int(i)
        tie = int(basis[g]) if rule == BLAND else g
        if (ratio, tie) < best[:2]:
            best = (ratio, tie, g)
    return best


def sharded_solve(T_loc, obj, basis, row0, allgather, rule="dantzig", eps_opt=1e-9,
                  eps_piv=1e-12, max_iters=0):
    """T_loc: this rank's constraint rows (m_local x N); obj: replicated
    objective row; allgather(np.ndarray) -> list of every rank's array.
    Mutates T_loc, obj, basis.  Returns (status, [(r, c), ...])."""
    N = obj.shape[0]
    m_local = T_loc.shape[0]
    hist = []
    while True:
        if max_iters and len(hist) >= max_iters:
            return ITER_LIMIT, hist
        c = select_entering(obj, N - 1, rule, eps_opt)
        if c is None:
            return OPTIMAL, hist
        k = local_key(T_loc, row0, c, basis, rule, eps_piv)
        pack = np.zeros(3 + N)
        pack[:3] = [k[0], float(k[1]), float(k[2])]
        if k[2] >= 0:
            rl = k[2] - row0
            pack[3:] = T_loc[rl, :] / T_loc[rl, c]
        packs = allgather(pack)
        w = min(range(len(packs)), key=lambda q: (float(packs[q][0]), int(packs[q][1])))
        if int(packs[w][2]) < 0:
            return UNBOUNDED, hist
        r = int(packs[w][2])
        p = packs[w][3:]
        rl = r - row0
        owner = 0 <= rl < m_local
        f = T_loc[:, c].copy()
        zc = obj[c]
        cols = np.flatnonzero(p != 0.0)
        pn = p[cols]
        T_loc[:, cols] = T_loc[:, cols] - np.multiply.outer(f, pn)
        obj[cols] = obj[cols] - zc * pn
        if owner:
            T_loc[rl, cols] = pn
        T_loc[:, c] = 0.0
        if owner:
            T_loc[rl, c] = 1.0
        obj[c] = 0.0
        basis[r] = c
        hist.append((r, c))


def _apply_slot(v, rows, j, slot, skip=True):
    """Pending pivot `slot` = (r_loc, c, f_loc, p) applied to values v at local
    rows `rows` of column j, or (rows scalar) at columns j of one row: the
    per-element rule of DESIGN.md §4b (apply_pivot in spx_delayed.hpp)."""
    r_loc, c, f_loc, p = slot
    rows = np.asarray(rows)
    j = np.asarray(j)
    pj = p[j]
    out = np.where(rows == r_loc, pj, v - f_loc[rows] * pj)
    if skip:
        out = np.where(pj == 0.0, v, out)
    return np.where(j == c, np.where(rows == r_loc, 1.0, 0.0), out)


def sharded_windowed_solve(T_loc, obj, basis, row0, allgather, K=8, rule="dantzig",
                           eps_opt=1e-9, eps_piv=1e-12, max_iters=0):
    """The row-sharded WINDOWED protocol (spx_delayed.hpp):
    the stored rows stay stale for up to K pivots; each pivot rebuilds the
    current pivot column (local rows) and this rank's candidate row from the
    stale values plus the pending slots, exchanges [key | current row / piv]
    in ONE all-gather, and the window is applied to the stored rows at the
    end (the flush).  Same signature and results as sharded_solve."""
    N = obj.shape[0]
    m_local = T_loc.shape[0]
    rows_all = np.arange(m_local)
    cols_all = np.arange(N)
    hist, pend = [], []

    def flush():
        for (r_loc, c, f_loc, p) in pend:  # the same element operations, in order
            cols = np.flatnonzero(p != 0.0)
            pn = p[cols]
            T_loc[:, cols] = T_loc[:, cols] - np.multiply.outer(f_loc, pn)
            if 0 <= r_loc < m_local:
                T_loc[r_loc, cols] = pn
            T_loc[:, c] = 0.0
            if 0 <= r_loc < m_local:
                T_loc[r_loc, c] = 1.0
        pend.clear()

    def current_col(j):
        v = T_loc[:, j].copy()
        for slot in pend:
            v = _apply_slot(v, rows_all, j, slot)
        return v

    def current_row(rl):
        v = T_loc[rl, :].copy()
        for slot in pend:
            v = _apply_slot(v, rl, cols_all, slot)
        return v

    while True:
        if max_iters and len(hist) >= max_iters:
            flush()
            return ITER_LIMIT, hist
        c = select_entering(obj, N - 1, rule, eps_opt)
        if c is None:
            flush()
            return OPTIMAL, hist
        f = current_col(c)
        b = current_col(N - 1)
        best = INF_KEY
        for i in np.flatnonzero(f > eps_piv):
            ratio = b[i] / f[i]
            if np.isnan(ratio):
                continue
            g = row0 + int(i)
            tie = int(basis[g]) if rule == BLAND else g
            if (ratio, tie) < best[:2]:
                best = (ratio, tie, g)
        pack = np.zeros(3 + N)
        pack[:3] = [best[0], float(best[1]), float(best[2])]
        if best[2] >= 0:
            rl = best[2] - row0
            pack[3:] = current_row(rl) / f[rl]
        packs = allgather(pack)
        w = min(range(len(packs)), key=lambda q: (float(packs[q][0]), int(packs[q][1])))
        if int(packs[w][2]) < 0:
            flush()
            return UNBOUNDED, hist
        r = int(packs[w][2])
        p = packs[w][3:].copy()
        zc = obj[c]
        cols = np.flatnonzero(p != 0.0)
        obj[cols] = obj[cols] - zc * p[cols]
        obj[c] = 0.0
        basis[r] = c
        hist.append((r, c))
        pend.append((r - row0, c, f, p))
        if len(pend) == K:
            flush()
