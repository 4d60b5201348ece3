"""The row_fix fold (round 6; spx_set_row_fix_fold, opt-in: it
measured no faster than a row_fix launch per window): a window's
fast-path leaving rows are rewritten inside the NEXT window's persistent chain
launch (each thread its own column, before the start handshake), and after a
call's last window by a gated row_fix.  Every result must
be BYTE-identical to the row_fix-per-window path and equal to the CPU oracle:
pivot sequence, basis, status and the tableau, also when fold windows meet
launch-per-phase windows, single pivots, forced pivots, start-handshake
aborts, the timed (event + graph) path and every reader of the tableau
between calls.
"""
import numpy as np
import pytest

from oracle import simplex_oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng_cls():
    from simplex_amd.engine import DeviceTableau
    return DeviceTableau


def _random_tableau(rows, cols, seed, zero_frac=0.1):
    rng = np.random.default_rng(seed)
    m = rows - 1
    n = max(1, cols - 1 - m)
    A = rng.uniform(0.05, 1.0, size=(m, n))
    A[rng.random(A.shape) < zero_frac] = 0.0
    T = np.zeros((m + 1, n + m + 1))
    T[:m, :n] = A
    T[np.arange(m), n + np.arange(m)] = 1.0
    T[:m, -1] = rng.uniform(1, 2, size=m) * n
    T[m, :n] = -rng.uniform(0.1, 1, size=n)
    return T, np.arange(n, n + m, dtype=np.int64)


def _oracle(T, basis, rule, k):
    ref, rb = T.copy(), basis.copy()
    st, hist = O.solve_tableau(ref, rb, rule=rule, max_iters=k)
    return st, hist, ref, rb


def _solve(eng_cls, T, basis, K, fold, rule, k, mode=2):
    with eng_cls(0) as e:
        e.set_window(K)
        e.set_chain(mode)
        e.set_row_fix_fold(fold)
        e.load(T, basis)
        res = e.solve(max_iters=k, rule=rule)
        return res, e.history().tolist(), e.tableau(), e.basis(), e.chain_blocks()


@pytest.mark.parametrize("K", [2, 4, 8, 16, 24, 28, 32])
@pytest.mark.parametrize("shape", [(17, 40), (300, 700), (1025, 2051)])
@pytest.mark.parametrize("rule", ["dantzig", "bland"])
def test_fold_matches_row_fix_per_window_and_oracle(eng_cls, K, shape, rule):
    T, basis = _random_tableau(*shape, seed=shape[0] * 5 + K, zero_frac=0.15)
    k = 5 * K + 3
    a = _solve(eng_cls, T, basis, K, True, rule, k)
    b = _solve(eng_cls, T, basis, K, False, rule, k)
    assert a[4] >= 1 and b[4] >= 1  # the persistent chain ran both times
    assert a[1] == b[1] and a[0].status == b[0].status and a[0].iters == b[0].iters
    assert a[2].tobytes() == b[2].tobytes() and np.array_equal(a[3], b[3])
    st, hist, ref, rb = _oracle(T, basis, rule, k)
    assert [tuple(x) for x in a[1]] == hist and a[0].status == st
    assert np.array_equal(a[2], ref) and np.array_equal(a[3], rb)


@pytest.mark.parametrize("K", [8, 24])
def test_fold_full_solves_with_negative_zeros(eng_cls, K):
    """Whole solves (every window a fold window, the last one's fix by the
    gated row_fix), with -0.0 entries and exact zeros (the flush's general
    path for ZERO columns, the fast path for the rest)."""
    T, basis = _random_tableau(600, 1500, seed=K, zero_frac=0.25)
    m = T.shape[0] - 1
    rng = np.random.default_rng(K + 1)
    blk = T[:m, :T.shape[1] - 1 - m]
    blk[rng.random(blk.shape) < 0.05] = -0.0
    a = _solve(eng_cls, T, basis, K, True, "dantzig", 0)
    b = _solve(eng_cls, T, basis, K, False, "dantzig", 0)
    assert a[0].status == 0 and a[1] == b[1] and a[2].tobytes() == b[2].tobytes()
    st, hist, ref, rb = _oracle(T, basis, "dantzig", 0)
    assert [tuple(x) for x in a[1]] == hist and np.array_equal(a[2], ref)


def test_fold_windows_meet_other_paths_on_one_context(eng_cls):
    """One context: fold windows through graphs (spx_run_pivots), a reader of
    the tableau, launch-per-phase windows (chain mode 1: the owed fix is
    settled before them), fold windows again, the fold switched off and on,
    single-pivot windows (spx_pivot), a forced pivot (spx_pivot_at), and a
    solve to the end -- the tableau equals the oracle's at every stop."""
    K = 8
    T, basis = _random_tableau(700, 1800, seed=3, zero_frac=0.1)
    ref, rb = T.copy(), basis.copy()
    done = []

    def oracle_to(k):
        nonlocal ref, rb
        st, h = O.solve_tableau(ref, rb, max_iters=k)
        done.extend(h)

    with eng_cls(0) as e:
        e.set_window(K)
        e.set_row_fix_fold(True)
        e.load(T, basis)
        steps = [("run", 4 * K + 3, 0), ("run", 2 * K, 1), ("run", 3 * K + 1, 0),
                 ("nofold", 2 * K, 0), ("run", 5 * K, 0), ("pivot", 3, 0), ("run", 2 * K + 5, 0)]
        for what, k, mode in steps:
            e.set_chain(mode)
            if what == "nofold":
                e.set_row_fix_fold(False)
                e.run_pivots(k)
                e.set_row_fix_fold(True)
            elif what == "pivot":
                for _ in range(k):
                    e.pivot()
            else:
                e.run_pivots(k)
            e.sync()
            oracle_to(k)
            assert [tuple(x) for x in e.history().tolist()] == done, what
            assert np.array_equal(e.tableau(), ref), what
            assert np.array_equal(e.basis(), rb), what
        # a forced pivot (spx_pivot_at) where the rules would pivot (so the
        # basis stays feasible), then 30 more windows
        c = O.select_entering(ref[-1], ref.shape[1] - 1, "dantzig", 1e-9)
        r = O.ratio_test(ref, c, rb, "dantzig", 1e-12)
        e.pivot_at(r, c)
        O.pivot(ref, r, c)
        rb[r] = c
        done.append((r, c))
        assert np.array_equal(e.tableau(), ref)
        res = e.solve(max_iters=30 * K)
        st, h = O.solve_tableau(ref, rb, max_iters=30 * K)
        done.extend(h)
        assert res.status == st
        assert [tuple(x) for x in e.history().tolist()] == done
        assert np.array_equal(e.tableau(), ref)


@pytest.mark.parametrize("K", [24, 32])
def test_fold_timed_graph_windows_bench_pattern(eng_cls, K):
    """bench.py's timed path: every 8th window launched directly between
    events, runs of 4 windows replayed from graphs captured for each window
    state, 20+ windows -- bit-exact with the oracle and the no-fold path."""
    T, basis = _random_tableau(1200, 4000, seed=K, zero_frac=0.05)
    outs = []
    for fold in (True, False):
        with eng_cls(0) as e:
            e.set_window(K)
            e.set_row_fix_fold(fold)
            e.load(T, basis)
            e.run_pivots(2 * K)          # warmup: builds the graphs
            e.sync()
            e.run_pivots(21 * K + 7, time_elim=8)
            e.sync()
            outs.append((e.history().tolist(), e.tableau()))
    assert outs[0][0] == outs[1][0] and outs[0][1].tobytes() == outs[1][1].tobytes()
    st, hist, ref, rb = _oracle(T, basis, "dantzig", 23 * K + 7)
    assert [tuple(x) for x in outs[0][0]] == hist and np.array_equal(outs[0][1], ref)


def test_fold_forced_handshake_aborts(eng_cls):
    """Every 3rd persistent window aborts at its start handshake (the test
    hook): its blocks have rewritten the owed rows before arriving, the
    aborted window owes nothing, and the rerun (launch-per-phase, after the
    gated row_fix, which rewrites the same values again) reads a settled
    tableau."""
    K = 8
    T, basis = _random_tableau(500, 1300, seed=11, zero_frac=0.1)
    with eng_cls(0) as e:
        e.set_window(K)
        e.set_row_fix_fold(True)
        e.set_chain_handshake(-3)
        e.load(T, basis)
        res = e.solve(max_iters=20 * K)
        h, out = e.history().tolist(), e.tableau()
        assert e.chain_reruns() > 0
    st, hist, ref, rb = _oracle(T, basis, "dantzig", 20 * K)
    assert [tuple(x) for x in h] == hist and res.status == st and np.array_equal(out, ref)


def test_fold_config3_width_first_windows(eng_cls):
    """The bench's shape class (config-3 width: 64 chain blocks, the RHS
    column riding along with the last thread, whose wave rewrites its leaving
    rows by lane) on fewer rows: 10 windows, fold vs no fold vs the oracle."""
    from simplex_amd import synth
    T, basis = synth.full_tableau("dense", 1024, 8192 + 8192 - 1024, 20251205)
    a = _solve(eng_cls, T, basis, 24, True, "dantzig", 240)
    b = _solve(eng_cls, T, basis, 24, False, "dantzig", 240)
    assert a[4] == 64 and a[1] == b[1] and a[2].tobytes() == b[2].tobytes()
    st, hist, ref, rb = _oracle(T, basis, "dantzig", 240)
    assert [tuple(x) for x in a[1]] == hist and np.array_equal(a[2], ref)
