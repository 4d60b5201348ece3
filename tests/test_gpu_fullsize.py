"""Full-size solves to optimality, pinned (BASELINE.json configs 3, 4, 5).

The fixtures (tests/golden/fullsize.json, fullsize_<config>.npz) come from the
C oracle (oracle/spx_oracle.c) run to optimality in the dev container by
tests/golden/make_fullsize.py, plus HiGHS (scipy linprog 'highs-ds', the
reference's answer path, solver_controller.py:76-85) on the same LP.  The GPU
solves the same LP through the C-ABI at the bench's window (K = 24) and must
reproduce EVERY pivot index, the final basis, the SHA-256 of the final tableau
bytes and the objective bit for bit, with the objective within 1e-9 relative of
HiGHS (north star tolerance).  Checkpoint digests along the way localise a
divergence.
"""
import hashlib
import json
import os
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")


def _fixture(name):
    path = os.path.join(GOLD, "fullsize.json")
    if not os.path.exists(path):
        pytest.skip("fullsize.json not generated")
    fx = json.load(open(path)).get(name)
    if not fx or "pivots" not in fx:
        pytest.skip(f"{name} fixture not generated")
    z = np.load(os.path.join(GOLD, f"fullsize_{name}.npz"))
    return fx, z["hist"].astype(np.int64), z["basis"].astype(np.int64)


def _digest(T):
    return hashlib.sha256(np.ascontiguousarray(T).tobytes()).hexdigest()


def _full_solve(name, window=24, chain=0):
    """The fixture's solve on the GPU: to optimality, or over the fixture's
    pivot prefix (max_pivots, status 1) when the oracle run was capped."""
    from simplex_amd import synth
    from simplex_amd.engine import DeviceTableau
    fx, hist, basis_end = _fixture(name)
    cap = fx.get("max_pivots", 0)
    Tf, obj, basis = synth.tableau_rows(fx["kind"], fx["m"], fx["n"], fx["seed"], order="F")
    with DeviceTableau(0) as e:
        e.set_window(window)
        e.set_chain(chain)
        e.load_rows(Tf, obj, basis, fx["m"], 0)
        del Tf
        done = 0
        for k in sorted(int(x) for x in fx["checkpoint_sha256"]):
            r = e.solve(rule=fx["rule"], max_iters=k - done)
            assert r.status == 1 and r.iters == k - done
            done = k
            assert _digest(e.tableau()) == fx["checkpoint_sha256"][str(k)], f"after {k} pivots"
        res = e.solve(rule=fx["rule"], max_iters=(cap - done) if cap else 0)
        h = e.history()
        assert res.status == fx["status"] == (1 if cap else 0)
        assert done + res.iters == fx["pivots"] == len(h)
        assert np.array_equal(h, hist), "pivot sequence differs from the oracle"
        assert np.array_equal(e.basis(), basis_end)
        z = res.objective
        assert z == fx["objective"], (z, fx["objective"])
        assert _digest(e.tableau()) == fx["tableau_sha256"]
    if fx.get("highs_status") == 0 and not cap:
        hz = fx["highs_objective"]
        assert abs(z - hz) <= 1e-9 * max(1.0, abs(hz)), (z, hz)
    return fx


@pytest.mark.parametrize("window,chain", [(24, 0), (28, 0), (32, 0), (16, 0), (24, 1), (0, 0)],
                         ids=["k24", "k28", "k32", "k16", "k24_launch_per_phase", "single_pivot"])
def test_config3_dantzig_full_solve_pinned(window, chain):
    """Config 3 (8192 x 8192 dense LP, tableau 8193 x 16385): the whole
    Dantzig solve vs the oracle's, index for index, at K = 16 / 24 / 28 / 32
    (the LEAN slot chains), with the launch-per-phase chain (mode 1), and one
    pivot per tableau pass (window 0)."""
    _full_solve("config3", window=window, chain=chain)


def test_config5_bland_100k_pivots_pinned():
    """Config 5 (4096 x 4096 degenerate LP, Bland): the first 100,000 pivots
    (Bland stalls at the degenerate origin far longer on this generator,
    profiles/r03/config5_bland_probe.log), every index and the tableau digests
    of the oracle's; the oracle's run revisits no basis (fixture)."""
    fx = _full_solve("config5")
    assert fx["basis_repeats"] == 0


@pytest.mark.parametrize("name", ["degen128", "degen256"])
def test_degenerate_bland_to_optimality_pinned(name):
    """The config-5 generator at 128 and 256 rows, where Bland terminates
    (7,604 and 56,262 pivots, almost all degenerate): to optimality, every
    index, the final tableau's digest, the objective within 1e-9 of HiGHS."""
    fx = _full_solve(name, window=8)
    assert fx["basis_repeats"] == 0


def test_config5_bland_million_pivots_pinned():
    """Config 5 over the 2^20 Bland pivots the GPU runs (K = 24): every index
    of the run against the C oracle's -- SHA-256 digests of the (r, c)
    sequence in 2^16-pivot chunks --, the tableau digests at 2^18, 2^19 and
    2^20 pivots, the final basis, and no basis revisited (Zobrist hashes of
    every basis along the run; the detector itself is checked on Beale's
    cycling LP in the CPU suite).  Fixture: make_fullsize.py config5long."""
    from simplex_amd import synth
    from simplex_amd.engine import DeviceTableau
    import sys
    sys.path.insert(0, GOLD)
    from make_fullsize import zobrist_repeats
    fx, hist, _ = _fixture("config5")
    if "long_hist_sha256" not in fx:
        pytest.skip("config5long fixture not generated")
    T, basis = synth.full_tableau("degenerate", 4096, 4096, 5)
    n, chunk = fx["long_pivots"], fx["long_chunk"]
    cps = {int(k): v for k, v in fx["long_checkpoint_sha256"].items()}
    with DeviceTableau(0) as e:
        e.set_window(24)
        e.load(T, basis)
        del T
        done = 0
        for k in sorted(cps):
            r = e.solve(rule="bland", max_iters=k - done)
            assert r.status == 1 and r.iters == k - done
            done = k
            assert _digest(e.tableau()) == cps[k], f"tableau after {k} pivots"
        assert done == n
        h = e.history()
        b = e.basis()
        z = e.state()[2]
    assert len(h) == n
    assert np.array_equal(h[:len(hist)], hist)
    for x, want in enumerate(fx["long_hist_sha256"]):
        got = hashlib.sha256(np.ascontiguousarray(h[x * chunk:(x + 1) * chunk],
                                                  dtype="<i8").tobytes()).hexdigest()
        assert got == want, f"pivots {x * chunk}..{(x + 1) * chunk - 1} differ from the oracle's"
    assert hashlib.sha256(np.ascontiguousarray(b.reshape(-1, 1), dtype="<i8").tobytes()
                          ).hexdigest() == fx["long_basis_sha256"]
    assert z == fx["long_objective"]
    assert zobrist_repeats(h, basis) == 0 == fx["long_basis_repeats"]


@pytest.mark.parametrize("window", [24, 28])
def test_config4_eight_virtual_ranks_240_pivots_pinned(window):
    """Config 4: the config-3 tableau row-sharded over 8 ranks (1024 rows
    each; virtual ranks on one GPU), 10 windows of 24 pivots: the pivot
    sequence is the oracle's and the assembled tableau matches the oracle's
    SHA-256 after 240 pivots (fixture checkpoint)."""
    from simplex_amd import dist, synth
    fx, hist, _ = _fixture("config3")
    m, n, k = fx["m"], fx["n"], 240
    world = 8
    uid = b"cfg4-240" + os.urandom(120)
    outs, errors = {}, []

    def rank_main(rank):
        try:
            r0, r1 = dist.row_partition(m, world, rank)
            Tl, obj, basis = synth.tableau_rows("dense", m, n, fx["seed"], r0, r1, order="F")
            with dist.ShardedTableau(0, rank, world, uid, local=True) as s:
                s.set_window(window)
                s.load_shard(Tl, obj, basis, m, r0)
                del Tl
                s.solve(max_iters=k)
                outs[rank] = (r0, r1, s.history(), s.tableau(), s.basis())
        except Exception as ex:  # pragma: no cover
            errors.append(ex)

    th = [threading.Thread(target=rank_main, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=900)
    assert not errors, errors
    for rank in range(world):
        assert np.array_equal(outs[rank][2], hist[:k])
        assert np.array_equal(outs[rank][3][-1], outs[0][3][-1])  # replicated objective row
        assert np.array_equal(outs[rank][4], outs[0][4])
    T = np.vstack([outs[r][3][:-1] for r in range(world)] + [outs[0][3][-1:]])
    assert _digest(T) == fx["checkpoint_sha256"][str(k)]
