"""The persistent pivot chain (spx_set_chain, csrc/spx_chain.hpp): one launch
runs a window's K pivot choices, with in-launch record exchanges instead of two
launches per pivot.  It must be BYTE-identical to the launch-per-phase chain
(mode 1) and to the single-pivot engine: pivot sequence, basis, status and the
tableau (tobytes), and np.array_equal to the CPU oracle.
"""
import os
import threading

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


def _run(eng_cls, T, basis, K, mode, min_blocks=0, **kw):
    with eng_cls(0) as e:
        e.set_window(K)
        e.set_chain(mode, min_blocks)
        e.load(T, basis)
        blocks = e.chain_blocks()
        res = e.solve(**kw)
        return res, e.history().tolist(), e.tableau(), e.basis(), blocks


@pytest.mark.parametrize("K", [2, 8, 16, 24, 28, 32])
@pytest.mark.parametrize("shape", [(2, 3), (17, 40), (300, 700), (1025, 2051)])
@pytest.mark.parametrize("rule", ["dantzig", "bland"])
@pytest.mark.parametrize("mode", [2, 3], ids=["cb256", "cb512"])
def test_chain_matches_lazy_chain_and_oracle(eng_cls, K, shape, rule, mode):
    T, basis = _random_tableau(*shape, seed=shape[0] * 7 + K)
    kw = dict(max_iters=3 * K + 5, rule=rule)
    res, h, out, b, blocks = _run(eng_cls, T, basis, K, mode, **kw)
    res1, h1, out1, b1, blocks1 = _run(eng_cls, T, basis, K, 1, **kw)
    assert blocks >= 1 and blocks1 == 0
    assert h == h1 and res.status == res1.status and res.iters == res1.iters
    assert out.tobytes() == out1.tobytes() and np.array_equal(b, b1)
    ref, rb = T.copy(), basis.copy()
    st, hist = O.solve_tableau(ref, rb, rule=rule, max_iters=3 * K + 5)
    assert [tuple(x) for x in h] == hist and res.status == st
    assert np.array_equal(out, ref) and np.array_equal(b, rb)


@pytest.mark.parametrize("mode", [2, 3], ids=["cb256", "cb512"])
@pytest.mark.parametrize("K", [2, 4, 8, 16, 24, 28, 32])
@pytest.mark.parametrize("shape", [(17, 40), (300, 700), (1025, 2051)])
@pytest.mark.parametrize("rule", ["dantzig", "bland"])
def test_chain_lean_slot_chains_with_negative_zeros_bit_exact(eng_cls, K, shape, rule, mode):
    """The LEAN slot chains (round 5: no per-slot guards, slots past q run as
    exact identities on +0 histories; used wherever the LDS histories fit and
    K % 4 == 0, the guarded chains otherwise: K = 2, and 512-thread blocks
    with K > 16) against the launch-per-phase chain and the oracle, with -0.0
    entries and exact zeros (the skip rule's masked paths) in the tableau."""
    T, basis = _random_tableau(*shape, seed=shape[0] * 13 + K, zero_frac=0.2)
    m = shape[0] - 1
    rng = np.random.default_rng(K)
    neg = rng.random((m, T.shape[1] - 1 - m)) < 0.05
    T[:m, :T.shape[1] - 1 - m][neg] = -0.0
    kw = dict(max_iters=3 * K + 5, rule=rule)
    res1, h1, out1, b1, _ = _run(eng_cls, T, basis, K, 1, **kw)
    res, h, out, b, blocks = _run(eng_cls, T, basis, K, mode, **kw)
    assert blocks >= 1
    assert h == h1 and res.status == res1.status and out.tobytes() == out1.tobytes()
    ref, rb = T.copy(), basis.copy()
    st, hist = O.solve_tableau(ref, rb, rule=rule, max_iters=3 * K + 5)
    assert [tuple(x) for x in h] == hist and np.array_equal(out, ref) and np.array_equal(b, rb)


@pytest.mark.parametrize("K", [4, 8])
def test_chain_512_threads_no_stale_entering_partials(eng_cls, K):
    """512-thread chain blocks: B = ceil((N-1)/512) blocks, but the window's
    first pivot reduces max(4 * ceil(N/256), B) entering partials.  Every
    window after the first must see only the previous chain's keys: here the
    most negative reduced costs sit in the upper column blocks (whose initial
    keys a stale partial would keep), so a stale key would re-pick a column
    that already entered (spx_chain.hpp)."""
    T, basis = _random_tableau(301, 2051, seed=91)
    n = 2051 - 1 - 300
    T[300, 1280:n] = -10.0 - 1e-3 * np.arange(n - 1280)
    kw = dict(max_iters=6 * K + 3)
    res, h, out, b, blocks = _run(eng_cls, T, basis, K, 3, **kw)
    assert blocks == 5
    ref, rb = T.copy(), basis.copy()
    st, hist = O.solve_tableau(ref, rb, max_iters=6 * K + 3)
    assert [tuple(x) for x in h] == hist and res.status == st
    assert np.array_equal(out, ref) and np.array_equal(b, rb)


@pytest.mark.parametrize("mode", [0])
@pytest.mark.parametrize("min_blocks", [0, 3, 64, 100, 256])
def test_chain_grid_sizes_bit_exact(eng_cls, min_blocks, mode):
    """More blocks than the minimum (fewer columns / rows per block, more than
    64 records per poll) give the same bytes."""
    T, basis = _random_tableau(400, 1300, seed=11 + min_blocks)
    res, h, out, b, blocks = _run(eng_cls, T, basis, 16, mode, min_blocks, max_iters=53)
    res1, h1, out1, b1, _ = _run(eng_cls, T, basis, 16, 1, max_iters=53)
    assert blocks == max(min_blocks, 6)
    assert h == h1 and res.iters == res1.iters and out.tobytes() == out1.tobytes()


def test_removed_chain_modes_rejected(eng_cls):
    """Round 4's one-XCD chains (modes 4 / 5) were slower than mode 0 on every
    same-box A/B and were removed in round 5: selecting one is
    an argument error, and the context keeps its chain."""
    from simplex_amd.engine import SpxError
    T, basis = _random_tableau(17, 40, seed=3)
    with eng_cls(0) as e:
        e.set_window(8)
        for mode in (4, 5, 6, -1):
            with pytest.raises(SpxError):
                e.set_chain(mode)
        e.load(T, basis)
        assert e.chain_blocks() >= 1


@pytest.mark.parametrize("mode,nb", [(0, 80), (2, 80), (3, 40)])
def test_chain_wide_tableau_more_than_64_blocks(eng_cls, mode, nb):
    """N > 64 x 256 columns: B = 80 blocks of 256 threads (two records per
    polling lane; the automatic choice), or 40 of 512."""
    T, basis = _random_tableau(301, 20400, seed=5)
    res, h, out, b, blocks = _run(eng_cls, T, basis, 24, mode, max_iters=60)
    assert blocks == nb
    res1, h1, out1, b1, _ = _run(eng_cls, T, basis, 24, 1, max_iters=60)
    assert h == h1 and out.tobytes() == out1.tobytes() and np.array_equal(b, b1)


@pytest.mark.parametrize("K", [8, 24])
@pytest.mark.parametrize("mode,nb", [(0, 64), (2, 64), (3, 32)])
def test_chain_config3_width_rhs_column_rides_along(eng_cls, K, mode, nb):
    """Config 3's width: N - 1 = 16384 candidate columns = 64 x 256, so the
    grid is 64 blocks (one record per polling lane) and the RHS column is kept
    by the last thread of the last block (spx_chain.hpp, xown): objective
    value, tag, p history and its flush record must match the lazy chain."""
    T, basis = _random_tableau(301, 16385, seed=8 + K)
    res, h, out, b, blocks = _run(eng_cls, T, basis, K, mode, max_iters=3 * K + 1)
    assert blocks == nb
    res1, h1, out1, b1, _ = _run(eng_cls, T, basis, K, 1, max_iters=3 * K + 1)
    assert h == h1 and res.status == res1.status and res.iters == res1.iters
    assert out.tobytes() == out1.tobytes() and np.array_equal(b, b1)
    ref, rb = T.copy(), basis.copy()
    st, hist = O.solve_tableau(ref, rb, max_iters=3 * K + 1)
    assert [tuple(x) for x in h] == hist and np.array_equal(out, ref)


@pytest.mark.parametrize("K", [4, 24, 32])
@pytest.mark.parametrize("mode", [0, 3])
def test_chain_degenerate_bland_full_solve(eng_cls, K, mode):
    from simplex_amd import synth
    T, basis = synth.full_tableau("degenerate", 96, 96, seed=3)
    res, h, out, b, _ = _run(eng_cls, T, basis, K, mode, rule="bland")
    res1, h1, out1, b1, _ = _run(eng_cls, T, basis, K, 1, rule="bland")
    ref, rb = T.copy(), basis.copy()
    st, hist = O.solve_tableau(ref, rb, rule="bland")
    assert res.status == res1.status == st == 0
    assert [tuple(x) for x in h] == hist == [tuple(x) for x in h1]
    assert out.tobytes() == out1.tobytes() and np.array_equal(out, ref)


def test_chain_stops_inside_window(eng_cls):
    """Optimal, unbounded and the iteration limit inside a window."""
    # optimal after a few pivots
    T, basis = _random_tableau(30, 80, seed=9)
    for mi in (0, 5, 13):
        r0 = _run(eng_cls, T, basis, 32, 0, max_iters=mi)
        r1 = _run(eng_cls, T, basis, 32, 1, max_iters=mi)
        assert r0[0].status == r1[0].status and r0[1] == r1[1]
        assert r0[2].tobytes() == r1[2].tobytes()
    # unbounded: a column with no positive entry enters
    T2, b2 = _random_tableau(20, 50, seed=4)
    n = 50 - 1 - 19
    T2[:19, 3] = -np.abs(T2[:19, 3]) - 0.1
    T2[19, 3] = -50.0
    r0 = _run(eng_cls, T2, b2, 8, 0)
    r1 = _run(eng_cls, T2, b2, 8, 1)
    ref, rb = T2.copy(), b2.copy()
    st, hist = O.solve_tableau(ref, rb)
    assert r0[0].status == r1[0].status == st == 3
    assert r0[1] == r1[1] == [list(x) for x in hist]
    assert r0[2].tobytes() == r1[2].tobytes()
    del n


def test_chain_resume_across_calls(eng_cls):
    """Several calls on one context (iteration limits mid-window, pivot_at)."""
    T, basis = _random_tableau(200, 600, seed=21)
    outs = []
    for mode in (0, 1):
        with eng_cls(0) as e:
            e.set_window(16)
            e.set_chain(mode)
            e.load(T, basis)
            e.solve(max_iters=7)
            e.solve(max_iters=20)
            e.pivot()
            e.solve(max_iters=30)
            outs.append((e.history().tolist(), e.tableau().tobytes(), e.basis().tolist()))
    assert outs[0] == outs[1]


def test_chain_concurrent_contexts(eng_cls):
    """Two contexts' persistent chains on two streams at once."""
    T, basis = _random_tableau(500, 1500, seed=33)
    res = [None, None]

    def work(k):
        res[k] = _run(eng_cls, T, basis, 24, 0, max_iters=100)

    th = [threading.Thread(target=work, args=(k,)) for k in range(2)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    ref = _run(eng_cls, T, basis, 24, 1, max_iters=100)
    for r in res:
        assert r[1] == ref[1] and r[2].tobytes() == ref[2].tobytes()


def test_chain_admission_more_chains_than_cus(eng_cls):
    """Six windowed contexts at config-3 width (64 chain blocks each: 384 >
    256 CUs) solving from six threads at once.  The process admits persistent
    chains only while their blocks fit the CUs; the others run the
    launch-per-phase chain.  Every context must finish byte-identical to a
    sequential run (no SPX_E_STATE from a partly resident chain)."""
    T, basis = _random_tableau(257, 16385, seed=61)
    kw = dict(max_iters=120)
    ref = _run(eng_cls, T, basis, 24, 0, **kw)
    assert ref[4] == 64
    res, stats, errs = [None] * 6, [None] * 6, []
    barrier = threading.Barrier(6)

    def work(k):
        try:
            with eng_cls(0) as e:
                e.set_window(24)
                e.load(T, basis)
                barrier.wait()
                for _ in range(3):  # several calls per context: admission per call
                    e.solve(max_iters=40)
                res[k] = (e.history().tolist(), e.tableau().tobytes())
                stats[k] = e.chain_stats()
        except Exception as ex:  # noqa: BLE001 - reported below
            errs.append(repr(ex))

    th = [threading.Thread(target=work, args=(k,)) for k in range(6)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errs, errs
    for r in res:
        assert r[0] == ref[1] and r[1] == ref[2].tobytes()
    assert sum(s["persistent_calls"] + s["refused_calls"] for s in stats) == 18
    assert all(s["blocks_held"] == 0 for s in stats)


def test_chain_budget_zero_runs_launch_per_phase(eng_cls):
    """spx_set_chain_budget(device, 0): every call is refused the persistent
    chain and runs the launch-per-phase chain, with the same bytes."""
    T, basis = _random_tableau(300, 900, seed=62)
    ref = _run(eng_cls, T, basis, 16, 0, max_iters=50)
    eng_cls.set_chain_budget(0, 0)
    try:
        with eng_cls(0) as e:
            e.set_window(16)
            e.load(T, basis)
            e.solve(max_iters=50)
            out, h, st = e.tableau(), e.history().tolist(), e.chain_stats()
    finally:
        eng_cls.set_chain_budget(0, -1)
    assert st["persistent_calls"] == 0 and st["refused_calls"] == 1
    assert h == ref[1] and out.tobytes() == ref[2].tobytes()
    with eng_cls(0) as e:  # default budget again: admitted
        e.set_window(16)
        e.load(T, basis)
        e.run_pivots(32)
        e.sync()
        assert e.chain_stats()["persistent_calls"] == 1


@pytest.mark.parametrize("mode", [0, 3])
def test_chain_handshake_forced_abort_reruns_bit_exact(eng_cls, mode):
    """spx_set_chain_handshake(ctx, -1): every persistent window aborts at its
    start handshake (ST_NOTRES) before any block stores anything; spx_solve,
    spx_pivot and spx_pivot_at rerun the aborted window with the
    launch-per-phase chain, so the bytes equal a plain run's and the oracle's.
    spx_run_pivots does not wait for its launches: the drain that follows it
    (spx_sync, spx_state, a getter) runs the missing pivots instead."""
    T, basis = _random_tableau(300, 900, seed=71)
    ref = _run(eng_cls, T, basis, 16, mode, max_iters=70)
    Tc, bc = T.copy(), basis.copy()
    O.solve_tableau(Tc, bc, max_iters=71)  # the 70 pivots + one rule-chosen pivot
    nb = set(bc.tolist())
    fc = next(j for j in range(T.shape[1] - 1) if j not in nb and abs(Tc[5, j]) > 0.05)
    O.pivot(Tc, 5, fc)
    bc[5] = fc
    with eng_cls(0) as e:
        e.set_window(16)
        e.set_chain(mode)
        e.load(T, basis)
        e.set_chain_handshake(-1)
        res = e.solve(max_iters=70)
        n0 = e.chain_reruns()
        assert n0 >= 1 and e.chain_blocks() > 0
        assert res.iters == ref[0].iters and e.history().tolist() == ref[1]
        assert e.tableau().tobytes() == ref[2].tobytes()
        e.pivot()
        e.pivot_at(5, fc)
        assert e.chain_reruns() >= n0 + 2
        assert np.array_equal(e.tableau(), Tc) and np.array_equal(e.basis(), bc)
        n2 = e.chain_reruns()
        e.run_pivots(40)
        e.sync()
        assert e.chain_reruns() == n2 + 1
        st, it, _ = e.state()
        assert it == 70 + 2 + 40
        O.solve_tableau(Tc, bc, max_iters=40)
        assert np.array_equal(e.tableau(), Tc) and np.array_equal(e.basis(), bc)
        e.run_pivots(16)  # no explicit sync: the next call's drain finishes it
        e.pivot()
        O.solve_tableau(Tc, bc, max_iters=17)
        assert e.state()[1] == 70 + 2 + 40 + 17
        assert np.array_equal(e.tableau(), Tc) and np.array_equal(e.basis(), bc)
        e.set_chain_handshake(0)  # automatic bound again: the next call runs persistent
        e.load(T, basis)
        n1 = e.chain_reruns()
        r2 = e.solve(max_iters=70)
        assert r2.iters == 70 and e.history().tolist() == ref[1]
        assert e.chain_stats()["persistent_calls"] >= 1
        assert e.chain_reruns() == n1  # every window ran persistent (no abort left behind)


def test_chain_handshake_more_chains_than_cus_without_admission(eng_cls):
    """Admission off (budget far above the CU count): six config-3-width chains
    (6 x 64 blocks > 256 CUs) from six threads.  A chain whose blocks are not
    all resident aborts at its start handshake before any store and the call
    reruns the window (launch-per-phase), instead of spinning into a fault:
    every context byte-identical to a sequential run, no SPX_E_STATE."""
    T, basis = _random_tableau(257, 16385, seed=63)
    kw = dict(max_iters=96)
    ref = _run(eng_cls, T, basis, 24, 0, **kw)
    assert ref[4] == 64
    res, reruns, errs = [None] * 6, [0] * 6, []
    barrier = threading.Barrier(6)

    def work(k):
        try:
            with eng_cls(0) as e:
                e.set_window(24)
                e.load(T, basis)
                barrier.wait()
                for _ in range(2):
                    e.solve(max_iters=48)
                res[k] = (e.history().tolist(), e.tableau().tobytes())
                reruns[k] = e.chain_reruns()
        except Exception as ex:  # noqa: BLE001 - reported below
            errs.append(repr(ex))

    eng_cls.set_chain_budget(0, 100000)
    try:
        th = [threading.Thread(target=work, args=(k,)) for k in range(6)]
        for x in th:
            x.start()
        for x in th:
            x.join()
    finally:
        eng_cls.set_chain_budget(0, -1)
    assert not errs, errs
    for r in res:
        assert r[0] == ref[1] and r[1] == ref[2].tobytes()
    print(f"windows rerun after a start-handshake abort: {sum(reruns)} ({reruns})")


_SHM_ENTRY = "<iiQ"  # {pid, blocks, start time}: 16 B, 64 entries (spx_capi.hip ShmEntry)


def _shm_entries(path):
    import fcntl
    import struct
    try:
        with open(path, "rb") as f:
            fcntl.flock(f, fcntl.LOCK_SH)
            raw = f.read(1024)
    except FileNotFoundError:
        return []
    raw = raw.ljust(1024, b"\0")
    return [struct.unpack_from(_SHM_ENTRY, raw, 16 * x)[:2] for x in range(64)]


def _proc_start(pid):
    """Field 22 of /proc/<pid>/stat (what libspx records with an entry)."""
    with open(f"/proc/{pid}/stat") as f:
        return int(f.read().rsplit(")", 1)[1].split()[19])


def _shm_put(path, pid, blocks, start=None):
    """Write an entry {pid, blocks, start} into a free slot of the admission
    table, under its flock (as another process's libspx would)."""
    import fcntl
    import struct
    start = _proc_start(pid) if start is None else start
    fd = os.open(path, os.O_RDWR | os.O_CREAT, 0o666)
    try:
        fcntl.flock(fd, fcntl.LOCK_EX)
        raw = os.pread(fd, 1024, 0).ljust(1024, b"\0")
        ent = [struct.unpack_from(_SHM_ENTRY, raw, 16 * x) for x in range(64)]
        slot = next(x for x, (p, b, _) in enumerate(ent) if p <= 0 or b <= 0)
        os.pwrite(fd, struct.pack(_SHM_ENTRY, pid, blocks, start), 16 * slot)
        fcntl.flock(fd, fcntl.LOCK_UN)
    finally:
        os.close(fd)


def test_chain_admission_shared_across_processes(eng_cls):
    """The admission budget is shared by the processes on a GPU through
    /dev/shm/spx_chain_<bus id> (the reference runs gunicorn with 2 workers,
    /root/reference/dockerfile:34).  Budget 256: with another live process
    holding 200 blocks, a 64-block chain is refused (launch-per-phase, same
    bytes); once that process is gone its entry is free and the chain is
    admitted; after spx_destroy (no explicit sync) this process's entry is 0."""
    import ctypes
    import subprocess
    from simplex_amd import _lib
    buf = ctypes.create_string_buffer(256)
    assert _lib.lib().spx_chain_shm_path(0, buf, 256) == 0
    path = buf.value.decode()
    assert path.startswith("/dev/shm/spx_chain_")
    T, basis = _random_tableau(65, 16385, seed=64)  # config-3 width: 64 chain blocks
    ref = _run(eng_cls, T, basis, 24, 0, max_iters=48)
    assert ref[4] == 64
    other = subprocess.Popen(["sleep", "300"])
    eng_cls.set_chain_budget(0, 256)
    try:
        _shm_put(path, other.pid, 200)
        with eng_cls(0) as e:
            e.set_window(24)
            e.load(T, basis)
            e.solve(max_iters=48)
            st = e.chain_stats()
            assert st["refused_calls"] == 1 and st["persistent_calls"] == 0, st
            assert e.history().tolist() == ref[1] and e.tableau().tobytes() == ref[2].tobytes()
            other.kill()
            other.wait()
            e.load(T, basis)
            e.solve(max_iters=48)
            assert e.chain_stats()["persistent_calls"] == 1
            assert not any(p == other.pid and b > 0 for p, b in _shm_entries(path))
            # an entry whose pid is alive but belongs to another process (a
            # reused pid: its start time differs) is stale too
            _shm_put(path, os.getppid(), 200, start=_proc_start(os.getppid()) + 12345)
            e.load(T, basis)
            e.solve(max_iters=48)
            assert e.chain_stats()["persistent_calls"] == 2
            assert not any(p == os.getppid() and b > 0 for p, b in _shm_entries(path))
            e.run_pivots(4 * 24)  # no sync: released behind the launches, or at destroy
        assert not any(p == os.getpid() and b > 0 for p, b in _shm_entries(path))
    finally:
        eng_cls.set_chain_budget(0, -1)
        if other.poll() is None:
            other.kill()
            other.wait()


def test_chain_admission_two_real_processes(tmp_path):
    """Two real libspx processes on GPU 0 (the reference's two gunicorn
    workers, /root/reference/dockerfile:34) share the admission table.  Budget
    24 blocks: the holder's 16-block chain is in flight (a long Bland run,
    enqueued without a sync), so the asker's 16-block chain does not fit and
    runs launch-per-phase; once the holder has exited, the asker's next call
    is admitted.  Both results equal each other and the oracle's."""
    import hashlib
    import json
    import subprocess
    import sys
    from simplex_amd import synth
    worker = os.path.join(os.path.dirname(os.path.abspath(__file__)), "adm_worker.py")
    sync = str(tmp_path)
    env = dict(os.environ)
    env.pop("SPX_CHAIN_SHM", None)
    env.pop("SPX_CHAIN_BUDGET", None)
    holder = subprocess.Popen([sys.executable, worker, "holder", sync, "24"], env=env,
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    asker = subprocess.Popen([sys.executable, worker, "asker", sync, "24"], env=env,
                             stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    try:
        hout, herr = holder.communicate(timeout=180)
        assert holder.returncode == 0, herr[-2000:]
        open(os.path.join(sync, "holder_done"), "w").close()
        aout, aerr = asker.communicate(timeout=180)
        assert asker.returncode == 0, aerr[-2000:]
    finally:
        for p_ in (holder, asker):
            if p_.poll() is None:
                p_.kill()
                p_.wait()
    h = json.loads(hout.strip().splitlines()[-1])
    a = json.loads(aout.strip().splitlines()[-1])
    assert h["stats"]["persistent_calls"] == 1, h
    st1, st2 = a["stats"]
    assert st1["refused_calls"] == 1 and st1["persistent_calls"] == 0, a
    assert st2["persistent_calls"] == 1, a
    assert a["iters"] == [48, 48] and a["digests"][0] == a["digests"][1]
    T, basis = synth.full_tableau("degenerate", 2048, 2048, 5)
    st, hist = O.solve_tableau(T, basis, rule="bland", max_iters=48)
    assert hashlib.sha256(np.asarray(hist, dtype=np.int64).tobytes()).hexdigest() == \
        a["digests"][0][0]
    assert hashlib.sha256(T.tobytes()).hexdigest() == a["digests"][0][1]


def test_chain_set_validated(eng_cls):
    with eng_cls(0) as e:
        with pytest.raises(Exception):
            e.set_chain(6)
        with pytest.raises(Exception):
            e.set_chain(0, 300)


@pytest.mark.parametrize("mode", [0, 1])
def test_chain_timing_events(eng_cls, mode):
    """spx_set_chain_timing: one event pair per window (persistent or lazy
    chain), same bytes as without the events."""
    T, basis = _random_tableau(300, 700, seed=17)
    with eng_cls(0) as e:
        e.set_window(8)
        e.set_chain(mode)
        e.load(T, basis)
        e.set_chain_timing(True)
        e.run_pivots(40)
        e.sync()
        ms, n = e.chain_timing(reset=True)
        assert n == 5 and ms > 0.0
        e.set_chain_timing(False)
        e.run_pivots(8)
        e.sync()
        assert e.chain_timing()[1] == 0
        out, h = e.tableau(), e.history().tolist()
    ref = _run(eng_cls, T, basis, 8, mode, max_iters=48)
    assert h == ref[1] and out.tobytes() == ref[2].tobytes()


@pytest.mark.parametrize("K", [8, 24])
@pytest.mark.parametrize("mode", [0, 3])
def test_chain_basic_columns_not_unit_vectors_at_load(eng_cls, K, mode):
    """Basic columns that are not exact unit vectors at load (a tiny entry, a
    -0.0, 1 + ulp) are ordinary data: the chain must not assume their values.
    Forced pivots on the affected rows make each of them the leaving row."""
    T, basis = _random_tableau(400, 1300, seed=40 + K)
    T[3, basis[7]] = 1e-300          # basic column of row 7 with an extra entry
    T[11, basis[2]] = -0.0           # -0.0 is not +0.0
    T[5, basis[5]] = 1.0 + 2.0 ** -52  # not exactly 1
    res, h, out, b, _ = _run(eng_cls, T, basis, K, mode, max_iters=3 * K + 3)
    res1, h1, out1, b1, _ = _run(eng_cls, T, basis, K, 1, max_iters=3 * K + 3)
    assert h == h1 and out.tobytes() == out1.tobytes() and np.array_equal(b, b1)
    ref, rb = T.copy(), basis.copy()
    st, hist = O.solve_tableau(ref, rb, max_iters=3 * K + 3)
    assert [tuple(x) for x in h] == hist and np.array_equal(out, ref)
    ref, rb = T.copy(), basis.copy()
    with eng_cls(0) as e:
        e.set_window(K)
        e.set_chain(mode)
        e.load(T, basis)
        for r in (3, 11, 5):
            nb = set(rb.tolist())
            c = next(j for j in range(T.shape[1] - 1) if j not in nb and abs(ref[r, j]) > 0.05)
            e.pivot_at(r, c)
            O.pivot(ref, r, c)
            rb[r] = c
        e.solve(max_iters=2 * K + 1)
        O.solve_tableau(ref, rb, max_iters=2 * K + 1)
        assert np.array_equal(e.tableau(), ref) and np.array_equal(e.basis(), rb)


def test_chain_after_single_pivots_on_the_same_context(eng_cls):
    """Single-pivot stretches and windows of different sizes on one context
    give the single-pivot engine's sequence and bytes."""
    T, basis = _random_tableau(300, 900, seed=77)
    with eng_cls(0) as e:
        e.set_window(0)
        e.load(T, basis)
        e.solve(max_iters=9)
        e.set_window(16)
        e.solve(max_iters=40)
        e.set_window(0)
        e.solve(max_iters=5)
        e.set_window(24)
        e.solve(max_iters=30)
        h, out = e.history().tolist(), e.tableau()
    with eng_cls(0) as e:
        e.set_window(0)
        e.load(T, basis)
        e.solve(max_iters=84)
        h0, out0 = e.history().tolist(), e.tableau()
    assert h == h0 and out.tobytes() == out0.tobytes()
