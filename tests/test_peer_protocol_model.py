"""CPU tests of the row-sharded persistent chain's cross-rank protocol
(tests/peer_protocol_model.py restates chain_shard_kernel + chain_start with a
thread per block and shared tagged granules).

The model must reproduce the oracle bit for bit under delays injected where
the GPU's timing varies (records published late, polls late, a rank running a
slot ahead), stop every rank at the same pivot on rank 0's stop bit, and rerun
a window whose start handshake aborted.  Two mutants show the protocol's
guards are load-bearing: one record half instead of two (by pivot parity)
deadlocks when a rank runs a slot ahead, and no window-end barrier lets a
rank's flush rewrite a row a peer is still gathering.
"""
import random
import threading

import numpy as np
import pytest

import peer_protocol_model as M
from oracle import simplex_oracle as O


def _run(world=2, B=2, kind="dense", m=20, n=14, seed=3, K=4, rule="dantzig", mutant=(),
         delay=None, late=None, max_iters=10 ** 6, hs_bound=0.5, stop_after=None, push=False,
         groups=None, late_rank=None):
    from simplex_amd import synth
    from simplex_amd.dist import row_partition
    dev = M.Device(world, B, mutant, push=push, groups=groups)
    ranks = []
    for r in range(world):
        r0, r1 = row_partition(m, world, r)
        T, obj, basis = synth.tableau_rows(kind, m, n, seed, r0, r1, order="C")
        lt = late_rank.get(r) if late_rank else late
        ranks.append(M.Rank(dev, r, T, obj, basis, r0, K, rule, delay=delay, late=lt,
                            hs_bound=hs_bound))
    errs, res = [], {}

    def go(rk):
        try:
            res[rk.rank] = rk.solve(max_iters)
        except Exception as ex:  # noqa: BLE001
            errs.append(ex)

    th = [threading.Thread(target=go, args=(rk,)) for rk in ranks]
    for t in th:
        t.start()
    if stop_after is not None:
        threading.Timer(stop_after, ranks[0].stop.set).start()
    for t in th:
        t.join()
    return ranks, res, errs


def _oracle(kind, m, n, seed, rule, max_iters=10 ** 6):
    from simplex_amd import synth
    T, basis = synth.full_tableau(kind, m, n, seed)
    st, hist = O.solve_tableau(T, basis, rule=rule, max_iters=max_iters)
    return st, hist, T, basis


def _check(ranks, res, kind, m, n, seed, rule, max_iters=10 ** 6):
    st, hist, T, basis = _oracle(kind, m, n, seed, rule, max_iters)
    for rk in ranks:
        assert res[rk.rank] == (st if len(hist) < max_iters else 1)
        assert rk.hist == hist
        r0 = rk.row0
        assert np.array_equal(rk.A, T[r0:r0 + rk.m_local])
        assert np.array_equal(rk.obj, T[-1])
        assert np.array_equal(rk.basis, basis)


def _jitter(seed, scale=2e-4):
    rng = random.Random(seed)
    lock = threading.Lock()

    def delay(*_):
        with lock:
            x = rng.random()
        if x < 0.3:
            import time
            time.sleep(x * scale / 0.3)
    return delay


@pytest.mark.parametrize("world,B,kind,m,n,K,rule", [
    (2, 2, "dense", 20, 14, 4, "dantzig"),
    (3, 2, "dense", 21, 16, 3, "dantzig"),
    (2, 3, "dense", 30, 25, 8, "dantzig"),
    (2, 2, "degenerate", 16, 16, 4, "bland"),
    (3, 3, "degenerate", 18, 18, 5, "bland"),
])
def test_model_matches_oracle_under_jitter(world, B, kind, m, n, K, rule):
    ranks, res, errs = _run(world, B, kind, m, n, 5, K, rule, delay=_jitter(world * 7 + K))
    assert not errs, errs
    _check(ranks, res, kind, m, n, 5, rule)


def test_model_rank_a_slot_ahead_is_safe_with_two_halves():
    """Rank 1 polls the ratio records late at every slot, so rank 0 publishes
    pivot q+1's records (into rank 1's buffer too) before rank 1 read pivot
    q's: the parity halves keep them apart."""
    import time

    def delay(point, rank, b, q, *rest):
        if point == "poll_ratio" and rank == 1:
            time.sleep(0.01)
    ranks, res, errs = _run(delay=delay)
    assert not errs, errs
    _check(ranks, res, "dense", 20, 14, 3, "dantzig")


def test_model_mutant_one_record_half_deadlocks():
    """The same schedule with ONE record buffer: rank 0's pivot-(q+1) records
    overwrite its pivot-q records in rank 1's buffer before rank 1 polled them,
    and rank 1's poll never matches (the kernels' ST_FAULT)."""
    import time

    def delay(point, rank, b, q, *rest):
        if point == "poll_ratio" and rank == 1 and q == 1:
            time.sleep(0.05)
    old = M.WAIT_LIMIT
    M.WAIT_LIMIT = 0.5
    try:
        _, _, errs = _run(delay=delay, mutant=("one_half",), max_iters=8)
    finally:
        M.WAIT_LIMIT = old
    assert errs and all(isinstance(e, M.Timeout) for e in errs), errs


def test_model_mutant_no_window_end_barrier_corrupts():
    """In the last slot of a window, a rank gathers the leaving row from its
    peer's rows late.  With the window-end barrier the owner's flush waits for
    it; without it the owner rewrites that row first and the late rank
    computes p from post-flush values."""
    import time

    K, m, n = 4, 40, 30

    def delay(point, rank, b, q, *rest):
        if point == "gather_row" and q == K - 1 and rest and rest[0] != rank:
            time.sleep(0.03)
    ranks, res, errs = _run(delay=delay, K=K, m=m, n=n)
    assert not errs, errs
    _check(ranks, res, "dense", m, n, 3, "dantzig")
    ranks, res, errs = _run(delay=delay, K=K, m=m, n=n, mutant=("no_done_barrier",))
    st, hist, T, basis = _oracle("dense", m, n, 3, "dantzig")
    broken = bool(errs) or any(rk.hist != hist or not np.array_equal(rk.A, T[rk.row0:rk.row0 + rk.m_local])
                               for rk in ranks)
    assert broken, "the no-barrier mutant reproduced the oracle: the schedule missed the hazard"


def test_model_stop_bit_stops_every_rank_at_the_same_pivot():
    """Rank 0's stop request rides in its ratio records: every rank stops
    before the same pivot, with the oracle's prefix."""
    import time

    def delay(*_):
        time.sleep(0.002)
    ranks, res, errs = _run(m=40, n=30, K=3, delay=delay, stop_after=0.05)
    assert not errs, errs
    its = {rk.it for rk in ranks}
    assert len(its) == 1
    k = its.pop()
    assert all(res[rk.rank] in (0, 1) for rk in ranks)
    _, hist, T, basis = _oracle("dense", 40, 30, 3, "dantzig", max_iters=k)
    for rk in ranks:
        assert rk.hist == hist
        assert np.array_equal(rk.A, T[rk.row0:rk.row0 + rk.m_local])


def test_model_start_handshake_late_block_aborts_then_reruns():
    """A block of rank 1 starts window 1 after the handshake bound: every
    block of every rank reads the same ABORT verdict, nothing is stored, each
    host reruns the window with the next epoch, and the solve is exact."""
    ranks, res, errs = _run(late=lambda W, b: 0.2 if W == 1 and b == 1 else 0.0,
                            hs_bound=0.05)
    assert not errs, errs
    assert all(rk.reruns >= 1 for rk in ranks)
    _check(ranks, res, "dense", 20, 14, 3, "dantzig")


def test_model_poll_geometry_covers_every_slot_up_to_512():
    """Wave 0's poll (64 lanes x RPL clamped records) reads every one of the
    nr * B ratio slots for every grid the shard geometry admits, up to config
    4's 8 ranks x 64 blocks = 512 = CHAIN_SH_SLOTS; one more is refused."""
    for br in (1, 2, 63, 64, 65, 128, 129, 256, 257, 320, 511, 512):
        assert M.poll_slots(br) == list(range(br))
    with pytest.raises(ValueError):
        M.poll_slots(513)


@pytest.mark.timeout(600)
@pytest.mark.parametrize("push", [False, True], ids=["pull", "push"])
def test_model_config4_geometry_8_ranks_64_blocks(push, monkeypatch):
    """Config 4's shard geometry: 8 ranks x 64 blocks, 512 ratio records per
    poll (the whole capacity, 8 records per polling lane), every record
    written into all 8 ranks' buffers, under jitter, and the leaving row
    gathered from its owner (pull) or pushed by it (push): the oracle's pivots,
    rows, objective row and basis, bit for bit (VERDICT r4 do-this 1)."""
    world, B, m, n, K, it = 8, 64, 64, 80, 4, 12
    # 512 block threads: poll with short sleeps so the spinning threads do
    # not starve the working ones of the GIL; a roomy handshake bound (the
    # threads of a window take a while to start)
    monkeypatch.setattr(M, "POLL_SLEEP", 2e-3)
    monkeypatch.setattr(M, "WAIT_LIMIT", 120.0)
    ranks, res, errs = _run(world, B, "dense", m, n, 11, K, "dantzig", max_iters=it,
                            delay=_jitter(97, scale=1e-4), push=push, hs_bound=30.0)
    assert not errs, errs
    assert all(rk.dev.slots == list(range(512)) for rk in ranks)
    _check(ranks, res, "dense", m, n, 11, "dantzig", max_iters=it)


@pytest.mark.parametrize("world,B,kind,m,n,K,rule", [
    (2, 2, "dense", 20, 14, 4, "dantzig"),
    (3, 3, "dense", 30, 25, 8, "dantzig"),
    (3, 2, "degenerate", 18, 18, 5, "bland"),
])
def test_model_push_matches_oracle_under_jitter(world, B, kind, m, n, K, rule):
    """Owner-push transport: the leaving row's owner writes its stale values
    into every peer's inbox; the result is the oracle's bit for bit."""
    ranks, res, errs = _run(world, B, kind, m, n, 5, K, rule, delay=_jitter(world * 11 + K),
                            push=True)
    assert not errs, errs
    _check(ranks, res, kind, m, n, 5, rule)


def test_model_push_needs_no_window_end_barrier():
    """The schedule that breaks the pull transport without its window-end
    barrier (a peer reads the owner's row after the owner's flush) is exact
    under push with no barrier at all: no peer ever reads another rank's rows.
    The inbox halves by pivot parity keep a rank that runs a slot ahead safe."""
    import time

    K, m, n = 4, 40, 30

    def delay(point, rank, b, q, *rest):
        if point == "gather_row" and q == K - 1 and rest and rest[0] != rank:
            time.sleep(0.03)
        if point == "poll_ratio" and rank == 1:
            time.sleep(0.002)
    ranks, res, errs = _run(delay=delay, K=K, m=m, n=n, push=True,
                            mutant=("no_done_barrier",))
    assert not errs, errs
    _check(ranks, res, "dense", m, n, 3, "dantzig")


# ---- device groups (ranks on different GPUs; round 6) -----------------------

@pytest.mark.parametrize("groups", [[0, 1], [0, 1, 2], [0, 0, 1]], ids=["2x1", "3x1", "2+1"])
def test_model_device_groups_bit_exact(groups):
    """Each device group settles its own start handshake, then waits for every
    other group's verdict (chain_start's cross-group stage): under jitter, with
    one to two ranks per group, every rank equals the oracle."""
    world = len(groups)
    ranks, res, errs = _run(world=world, B=2, m=24, n=16, seed=5, K=4, groups=groups,
                            delay=_jitter(11))
    assert not errs, errs
    _check(ranks, res, "dense", 24, 16, 5, "dantzig")


def _late_first_window(seconds):
    def late(W, b):
        return seconds if W == 1 else 0.0
    return late


def test_model_late_device_group_is_aborted_by_cas():
    """A group whose ranks reach the first window later than the spin bound
    (WAIT_LIMIT, the kernels' ~4 s; here 6 s): the early group, having said
    GO, decides the late group's window ABORT by CAS once the handshake bound
    passed, and both rerun until the late one catches up -- bit-exact, with
    reruns on every rank.  Without the CAS (mutant), the early group's wait
    runs into the bound (the round-5 ST_FAULT)."""
    kw = dict(world=2, B=2, m=20, n=14, seed=3, K=4, groups=[0, 1], hs_bound=0.2,
              late_rank={1: _late_first_window(6.0)})
    ranks, res, errs = _run(**kw)
    assert not errs, errs
    _check(ranks, res, "dense", 20, 14, 3, "dantzig")
    assert all(rk.reruns > 0 for rk in ranks), [rk.reruns for rk in ranks]
    ranks, res, errs = _run(mutant=("no_group_cas",), **kw)
    assert errs and all(isinstance(e, M.Timeout) for e in errs), errs
