"""Synthetic LP generators for the benchmark configs (BASELINE.json configs 2-5).

Every element is a pure function of (seed, stream, index) — splitmix64 of a
mixed 64-bit counter — so any rank can generate exactly its own row block
of the tableau without generating (or communicating) the rest, and the same
numbers come out at every world size.

dense_lp  (configs 2-4): standard-form MAX, all rows "<=", b > 0, so the
  slack basis is feasible (phase 2 only) and A > 0 keeps it bounded:
    A[i,j] = 0.1 + 0.9*u(seed, 0, i*n + j)
    b[i]   = (1 + u(seed, 1, i)) * n / 4
    c[j]   = 0.1 + 0.9*u(seed, 2, j)
degenerate_lp (config 5, Bland): integer data with exact ratio ties:
    rows i < m-1, i even: A in {-4..4}, b = 0
    rows i < m-1, i odd : A in {1..9},  b = 1
    row m-1             : sum(x) <= 10 n (boundedness)
    c in {1..9}
Tableau: [A | I | b] with objective row [-c | 0 | 0] last, basis = slacks.
"""
from __future__ import annotations

import numpy as np

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)
_G = np.uint64(0x9E3779B97F4A7C15)
_S = np.uint64(0xD1B54A32D192ED03)
_C1 = np.uint64(0xBF58476D1CE4E5B9)
_C2 = np.uint64(0x94D049BB133111EB)


def _mix(seed: int, stream: int, idx: np.ndarray) -> np.ndarray:
    """splitmix64 finaliser of seed*G + stream*S + idx (mod 2^64)."""
    with np.errstate(over="ignore"):
        x = (np.uint64(seed) * _G + np.uint64(stream) * _S) + idx.astype(np.uint64)
        z = x + _G
        z = (z ^ (z >> np.uint64(30))) * _C1
        z = (z ^ (z >> np.uint64(27))) * _C2
        z = z ^ (z >> np.uint64(31))
    return z


def uniform(seed: int, stream: int, idx: np.ndarray) -> np.ndarray:
    """Doubles in [0, 1) with 53 random bits."""
    z = _mix(seed, stream, idx)
    return (z >> np.uint64(11)).astype(np.float64) * (2.0 ** -53)


def _ints(seed: int, stream: int, idx: np.ndarray, lo: int, hi: int) -> np.ndarray:
    z = _mix(seed, stream, idx)
    return (z % np.uint64(hi - lo + 1)).astype(np.int64) + lo


def dense_lp(m: int, n: int, seed: int, row0: int = 0, row1: int | None = None):
    """(A_block (rows x n), b_block, c) of the dense random-feasible LP."""
    row1 = m if row1 is None else row1
    rows = np.arange(row0, row1, dtype=np.uint64)
    idx = rows[:, None] * np.uint64(n) + np.arange(n, dtype=np.uint64)[None, :]
    A = 0.1 + 0.9 * uniform(seed, 0, idx)
    b = (1.0 + uniform(seed, 1, rows)) * (n / 4.0)
    c = 0.1 + 0.9 * uniform(seed, 2, np.arange(n, dtype=np.uint64))
    return A, b, c


def degenerate_lp(m: int, n: int, seed: int, row0: int = 0, row1: int | None = None):
    row1 = m if row1 is None else row1
    rows = np.arange(row0, row1, dtype=np.int64)
    idx = rows.astype(np.uint64)[:, None] * np.uint64(n) + np.arange(n, dtype=np.uint64)[None, :]
    mixed = _ints(seed, 0, idx, -4, 4).astype(np.float64)
    pos = _ints(seed, 3, idx, 1, 9).astype(np.float64)
    even = (rows % 2 == 0)[:, None]
    A = np.where(even, mixed, pos)
    b = np.where(rows % 2 == 0, 0.0, 1.0)
    last = rows == m - 1
    A[last] = 1.0
    b[last] = 10.0 * n
    c = _ints(seed, 2, np.arange(n, dtype=np.uint64), 1, 9).astype(np.float64)
    return A, b, c


def tableau_rows(kind: str, m: int, n: int, seed: int, row0: int = 0, row1: int | None = None,
                 order: str = "F"):
    """This rank's constraint rows of the slack-basis tableau [A | I | b].

    Returns (T_rows (row1-row0) x N in `order`, obj (N,), basis (m,)), where
    N = n + m + 1 and obj = [-c | 0 | 0].
    """
    row1 = m if row1 is None else row1
    gen = {"dense": dense_lp, "degenerate": degenerate_lp}[kind]
    A, b, c = gen(m, n, seed, row0, row1)
    N = n + m + 1
    T = np.zeros((row1 - row0, N), dtype=np.float64, order=order)
    T[:, :n] = A
    T[np.arange(row1 - row0), n + np.arange(row0, row1)] = 1.0
    T[:, N - 1] = b
    obj = np.zeros(N, dtype=np.float64)
    obj[:n] = -c
    basis = np.arange(n, n + m, dtype=np.int64)
    return T, obj, basis


def full_tableau(kind: str, m: int, n: int, seed: int) -> tuple:
    """Whole (m+1) x N row-major tableau (objective row last) and basis."""
    T, obj, basis = tableau_rows(kind, m, n, seed, order="C")
    return np.vstack([T, obj[None, :]]), basis


def lp_data(kind: str, m: int, n: int, seed: int):
    """(A, b, c) of the whole LP (for HiGHS cross-checks)."""
    gen = {"dense": dense_lp, "degenerate": degenerate_lp}[kind]
    return gen(m, n, seed)
