"""Windowed ("delayed") elimination (spx_set_window, csrc/spx_delayed.hpp):
K pivots per streaming pass over the tableau must be bit-identical to K
single-pivot passes, and both to the CPU oracle.

Bar: pivot sequence, basis and status identical; tableau BYTE-identical to the
single-pivot engine (tobytes, so even the sign of zero) and np.array_equal to
the oracle.
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


def _run(eng_cls, T, basis, K, **kw):
    with eng_cls(0) as e:
        e.set_window(K)
        e.load(T, basis)
        res = e.solve(**kw)
        return res, e.history().tolist(), e.tableau(), e.basis()


@pytest.mark.parametrize("K", [2, 8, 12, 16, 24, 28, 32])
@pytest.mark.parametrize("shape", [(2, 3), (17, 40), (300, 700), (1025, 2051)])
@pytest.mark.parametrize("skip", [True, False], ids=["skip", "dense"])
def test_window_rule_pivots_bit_exact(eng_cls, K, shape, skip):
    T, basis = _random_tableau(*shape, seed=shape[0] * 7 + shape[1])
    ref, rb = T.copy(), basis.copy()
    st, hist = O.solve_tableau(ref, rb, max_iters=37, skip_zero=skip)
    res, h, out, b = _run(eng_cls, T, basis, K, max_iters=37, skip_zero_cols=skip)
    res0, h0, out0, b0 = _run(eng_cls, T, basis, 0, max_iters=37, skip_zero_cols=skip)
    assert [tuple(x) for x in h] == hist and h == h0
    assert res.status == res0.status == st and res.iters == res0.iters == len(hist)
    assert np.array_equal(out, ref) and np.array_equal(b, rb)
    assert out.tobytes() == out0.tobytes()


def _set_flush_map(e, fmap):
    """fmap = flush block map (bit 0 chunk-major, bit 1 groups rotated by chunk)."""
    e.set_elim_variant(0, 0, -1, flush_map=fmap)
    v = e.elim_variant()
    assert (v["flush_var"], v["flush_map"]) == (0, fmap)


@pytest.mark.parametrize("fmap", [0, 1, 2, 3])
@pytest.mark.parametrize("K", [2, 12, 16, 24, 28, 32])
@pytest.mark.parametrize("shape", [(17, 40), (700, 1500), (1537, 2600)])
def test_window_flush_block_maps_bit_exact(eng_cls, fmap, K, shape):
    """The LDS-DMA flush under every block map (group-major, chunk-major,
    rotated groups) gives the single-pivot bytes."""
    T, basis = _random_tableau(*shape, seed=shape[0] + 3 * shape[1] + fmap)
    with eng_cls(0) as e:
        e.set_window(K)
        e.load(T, basis)
        _set_flush_map(e, fmap)
        res = e.solve(max_iters=3 * K + 5)
        h, out = e.history().tolist(), e.tableau()
    with eng_cls(0) as s:
        s.load(T, basis)
        res0 = s.solve(max_iters=3 * K + 5)
        assert h == s.history().tolist()
        assert res.status == res0.status and res.iters == res0.iters
        assert out.tobytes() == s.tableau().tobytes()


def test_removed_flush_variants_rejected(eng_cls):
    """The register-ring (1-5), ring-9/10 (6/7) and dynamically claimed flushes
    measured slower and were removed: selecting one is an error."""
    with eng_cls(0) as e:
        for fv in (1, 5, 6, 7):
            with pytest.raises(Exception):
                e.set_elim_variant(0, 0, -1, flush_variant=fv)
        with pytest.raises(Exception):
            e.set_elim_variant(0, 0, -1, flush_map=4)


@pytest.mark.parametrize("K", [4, 16])
def test_window_config2_full_solve(eng_cls, K):
    """BASELINE config 2 (1024 x 2048): every pivot, final tableau, objective."""
    from simplex_amd import synth
    T, basis = synth.full_tableau("dense", 1024, 2048, 20251207)
    ref, rb = T.copy(), basis.copy()
    st, hist = O.solve_tableau(ref, rb)
    res, h, out, b = _run(eng_cls, T, basis, K)
    assert res.status == st == 0 and res.iters == len(hist)
    assert [tuple(x) for x in h] == hist
    assert np.array_equal(out, ref) and np.array_equal(b, rb)
    assert res.objective == ref[-1, -1]


@pytest.mark.parametrize("K", [4, 32])
def test_window_degenerate_bland(eng_cls, K):
    """Bland on a degenerate LP: ratio ties by basis index inside a window read
    the basis as updated by the window's earlier pivots."""
    from simplex_amd import synth
    T, basis = synth.full_tableau("degenerate", 96, 96, 9)
    ref, rb = T.copy(), basis.copy()
    seen = []
    st, hist = O.solve_tableau(ref, rb, rule="bland", max_iters=100000,
                               on_pivot=lambda r, c, _T: seen.append(rb.copy()))
    assert st == 0
    with eng_cls(0) as e:
        e.set_window(K)
        e.load(T, basis)
        for k in range(min(20, len(hist))):  # single pivots: windows of one
            assert e.pivot(rule="bland") == hist[k]
            assert np.array_equal(e.basis(), seen[k])
        res = e.solve(rule="bland")
        assert res.status == 0
        assert [tuple(x) for x in e.history().tolist()] == hist
        assert np.array_equal(e.tableau(), ref) and np.array_equal(e.basis(), rb)


@pytest.mark.parametrize("K", [4, 8])
def test_window_iteration_limit_mid_window_and_resume(eng_cls, K):
    """A limit that falls inside a window stops there; resuming continues the
    same sequence (the window's unmade slots leave the tableau alone)."""
    from simplex_amd import synth
    T, basis = synth.full_tableau("dense", 64, 96, 7)
    with eng_cls(0) as a, eng_cls(0) as b:
        a.set_window(K)
        a.load(T, basis)
        b.load(T, basis)
        for lim in (5, 1, 3):
            r1 = a.solve(max_iters=lim)
            assert r1.status == 1 and r1.iters == lim
        r2 = a.solve()
        rb = b.solve()
        assert r2.status == rb.status == 0 and 9 + r2.iters == rb.iters
        assert a.history().tolist() == b.history().tolist()
        assert a.tableau().tobytes() == b.tableau().tobytes()


def test_window_unbounded_and_optimal_stop_inside_window(eng_cls):
    """Terminal states reached mid-window: nothing after them is applied."""
    # unbounded: x1 enters with no positive entry in its column
    T = np.array([[-1.0, 1.0, 1.0, 0.0, 2.0],
                  [-1.0, 0.0, 0.0, 1.0, 3.0],
                  [-1.0, -2.0, 0.0, 0.0, 0.0]])
    basis = np.array([2, 3], dtype=np.int64)
    ref, rb = T.copy(), basis.copy()
    st, hist = O.solve_tableau(ref, rb)
    res, h, out, b = _run(eng_cls, T, basis, 8)
    assert res.status == st == 3
    assert [tuple(x) for x in h] == hist
    assert np.array_equal(out, ref) and np.array_equal(b, rb)
    # optimal after 2 pivots of a 16-window
    T, basis = _random_tableau(4, 9, seed=3)
    ref, rb = T.copy(), basis.copy()
    st, hist = O.solve_tableau(ref, rb)
    res, h, out, b = _run(eng_cls, T, basis, 16)
    assert res.status == st == 0 and [tuple(x) for x in h] == hist
    assert np.array_equal(out, ref)


def test_window_forced_pivots_and_two_phase(eng_cls):
    """spx_pivot_at (drive-out of artificials) in window mode, and the host
    two-phase driver over a windowed engine."""
    T, basis = _random_tableau(40, 100, seed=5, zero_frac=0.0)
    ref = T.copy()
    with eng_cls(0) as e:
        e.set_window(8)
        e.load(T, basis)
        for r, c in ((3, 7), (10, 2), (3, 0)):
            e.pivot_at(r, c)
            O.pivot(ref, r, c, skip_zero=True)
            assert np.array_equal(e.tableau(), ref)
    from simplex_amd import lp
    rows = [([1.0, 1.0, 1.0], "<=", 40.0), ([2.0, 1.0, -1.0], ">=", 10.0),
            ([0.0, -1.0, 1.0], ">=", 10.0), ([1.0, 0.0, 1.0], "=", 25.0)]
    sf = lp.build_standard_form([2.0, 3.0, 4.0], rows, maximize=True)
    assert sf.k > 0  # phase 1 + drive-out needed

    def windowed():
        w = eng_cls(0)
        w.set_window(8)
        return w

    r0 = lp.solve_standard_form(sf)
    r8 = lp.solve_standard_form(sf, engine_factory=windowed)
    assert r0.status == r8.status == 0 and r0.objective == r8.objective
    assert np.array_equal(r0.x, r8.x) and r0.pivots == r8.pivots


@pytest.mark.parametrize("K", [4, 16])
def test_window_timed_graph_and_chunks(eng_cls, K):
    """bench.py's timed region in window mode: event pairs around every flush;
    graph replay, direct launches and a ragged remainder all agree."""
    from simplex_amd import synth
    T, basis = synth.full_tableau("dense", 300, 500, 21)
    outs = []
    for kw in (dict(time_elim=1, use_graph=True), dict(time_elim=1, use_graph=False),
               dict(time_elim=0, use_graph=True), dict(time_elim=0, use_graph=False)):
        with eng_cls(0) as e:
            e.set_window(K)
            e.load(T, basis)
            e.run_pivots(5)
            e.sync()
            e.elim_timing(reset=True)
            e.run_pivots(41, **kw)
            e.sync()
            ms, cnt, cols = e.elim_timing(reset=True)
            if kw["time_elim"]:
                assert cnt == -(-41 // K) and ms > 0 and cols > 0
            outs.append((e.history().tolist(), e.tableau()))
    for h, t in outs[1:]:
        assert h == outs[0][0] and t.tobytes() == outs[0][1].tobytes()
    ref, rb = T.copy(), basis.copy()
    st, hist = O.solve_tableau(ref, rb, max_iters=46)
    assert [tuple(x) for x in outs[0][0]] == hist and np.array_equal(outs[0][1], ref)


@pytest.mark.parametrize("pad", [0, 2, 130, 1024])
def test_window_ld_padding_and_odd_rows(eng_cls, pad):
    from simplex_amd import synth
    T, basis = synth.full_tableau("dense", 257, 300, 4)
    with eng_cls(0) as e, eng_cls(0) as s:
        e.set_ld_pad(pad)
        e.set_window(16)
        e.load(T, basis)
        s.load(T, basis)
        r = e.solve()
        r0 = s.solve()
        assert r.iters == r0.iters and e.history().tolist() == s.history().tolist()
        assert e.tableau().tobytes() == s.tableau().tobytes()


def test_window_sizes_validated(eng_cls):
    with eng_cls(0) as e:
        for bad in (3, 5, 10, 20, 30, 33, 64, -1):
            with pytest.raises(Exception):
                e.set_window(bad)
        for good in (0, 1, 2, 4, 8, 12, 16, 24, 28, 32):
            e.set_window(good)


@pytest.mark.parametrize("world,kind,m,n,rule,K", [
    (2, "dense", 200, 300, "dantzig", 8),
    (3, "dense", 301, 257, "dantzig", 24),
    (4, "dense", 1024, 2048, "dantzig", 16),
    (2, "degenerate", 64, 64, "bland", 12),
    (5, "dense", 7, 9, "dantzig", 4),   # ranks with one or two rows
])
def test_window_sharded_virtual_ranks_bit_exact(world, kind, m, n, rule, K):
    """Row-sharded windows (lazy_prep -> all-gather of [key | current row] ->
    lazy_norm FINISH per pivot, a local flush per window) through the
    in-process exchange: every rank's rows, objective row, basis and pivot
    sequence equal the oracle's full solve."""
    from simplex_amd import synth
    from test_gpu_engine import _sharded_threads
    outs = _sharded_threads(world, kind, m, n, 3, rule, window=K)
    T, basis = synth.full_tableau(kind, m, n, 3)
    st, hist = O.solve_tableau(T, basis, rule=rule, max_iters=200000)
    for rank, (r0, r1, res, h, Tl, b) in outs.items():
        assert res.status == st
        assert [tuple(x) for x in h] == hist
        assert np.array_equal(Tl[:-1], T[r0:r1])
        assert np.array_equal(Tl[-1], T[-1])
        assert np.array_equal(b, basis)


def test_window_sharded_single_rank_rccl_matches_plain(eng_cls):
    """A 1-rank RCCL communicator runs the sharded window protocol (prep,
    ncclAllGather, FINISH) inside the captured window graph: byte-identical
    to the plain windowed engine."""
    from simplex_amd import dist
    T, basis = _random_tableau(300, 700, seed=17)
    with eng_cls(0) as e:
        e.set_window(16)
        e.load(T, basis)
        e.solve(max_iters=70)
        h0, t0 = e.history().tolist(), e.tableau()
    with dist.ShardedTableau(0, 0, 1, dist.make_unique_id()) as s:
        s.set_window(16)
        s.load(T, basis)
        s.solve(max_iters=70)
        assert s.history().tolist() == h0
        assert s.tableau().tobytes() == t0.tobytes()


@pytest.mark.parametrize("K", [16, 24])
def test_window_config3_size_matches_single_pivot_path(eng_cls, K):
    """8192 x 16385 (BASELINE config 3): 48 pivots in K-windows (K = 24, the
    bench default: a 3-pivot call, then 45 = one full window and a partial
    one) are byte-identical to 48 single-pivot passes; first 3 vs the oracle."""
    from simplex_amd import synth
    m = n = 8192
    Tf, obj, basis = synth.tableau_rows("dense", m, n, 20251205, order="F")
    with eng_cls(0) as e:
        e.set_window(K)
        e.load_rows(Tf, obj, basis, m, 0)
        T = np.vstack([np.ascontiguousarray(Tf), obj[None, :]])
        rb = basis.copy()
        st, hist = O.solve_tableau(T, rb, max_iters=3)
        e.solve(max_iters=3)
        assert [tuple(h) for h in e.history().tolist()] == hist
        assert np.array_equal(e.tableau(), T)
        del T
        e.solve(max_iters=45)
        hw, tw = e.history().tolist(), e.tableau()
    with eng_cls(0) as s:
        s.load_rows(Tf, obj, basis, m, 0)
        del Tf
        s.solve(max_iters=48)
        assert s.history().tolist() == hw
        assert s.tableau().tobytes() == tw.tobytes()


def test_two_phase_driver_auto_window_matches_single_pivot():
    """lp.solve_standard_form picks K-pivot windows by size (auto_window: 8 at
    this ~1.3M-cell tableau); phase 1, drive-out and phase 2 give the exact
    pivot sequence, point and objective of the single-pivot engine."""
    from simplex_amd import lp
    from simplex_amd.engine import auto_window
    rng = np.random.default_rng(11)
    m, n = 600, 1300
    rows = []
    for i in range(m):
        a = rng.uniform(0.05, 1.0, size=n)
        a[rng.random(n) < 0.2] = 0.0
        if i % 7 == 0:
            rows.append((a.tolist(), ">=", float(rng.uniform(1, 5))))
        elif i % 11 == 0:
            rows.append((a.tolist(), "=", float(rng.uniform(20, 40))))
        else:
            rows.append((a.tolist(), "<=", float(rng.uniform(50, 100))))
    c = rng.uniform(0.1, 1.0, size=n).tolist()
    sf = lp.build_standard_form(c, rows, maximize=True)
    assert sf.k > 0 and auto_window(sf.m, sf.N) == 8
    r_auto = lp.solve_standard_form(sf)
    r_one = lp.solve_standard_form(sf, window=0)
    assert r_auto.status == r_one.status
    assert r_auto.pivots == r_one.pivots and r_auto.iters == r_one.iters
    if r_one.status == 0:
        assert r_auto.objective == r_one.objective
        assert np.array_equal(r_auto.x, r_one.x)


@pytest.mark.parametrize("tail", ["0", "10", "30", "50"])
@pytest.mark.parametrize("K", [8, 24])
@pytest.mark.parametrize("shape", [(17, 40), (700, 1500), (1537, 2600)])
def test_window_flush_tail_split_bit_exact(eng_cls, monkeypatch, tail, K, shape):
    """The flush's record split with a tail share (SPX_FLUSH_TAIL, read at
    context creation: the last x % of the record rows go to the first two
    dispatch rounds' groups).  Only which wave updates a column changes, so the
    bytes are the single-pivot path's."""
    T, basis = _random_tableau(*shape, seed=shape[0] + 5 * shape[1] + K)
    monkeypatch.setenv("SPX_FLUSH_TAIL", tail)
    res, h, out, b = _run(eng_cls, T, basis, K, max_iters=3 * K + 5)
    monkeypatch.delenv("SPX_FLUSH_TAIL")
    res0, h0, out0, b0 = _run(eng_cls, T, basis, 0, max_iters=3 * K + 5)
    assert h == h0 and res.status == res0.status and res.iters == res0.iters
    assert out.tobytes() == out0.tobytes() and np.array_equal(b, b0)
