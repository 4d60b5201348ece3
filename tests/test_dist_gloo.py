"""World-size-2 (and 3) gloo tests of the row-sharded path on CPU.

Covers the host side of simplex_amd.dist (row partition, RCCL unique-id
exchange through torch.distributed) and the per-pivot exchange protocol that
libspx runs over RCCL, one all-gather of [leaving key | normalised row] per
pivot (oracle/sharded_oracle.py restates it with gloo collectives): the
sharded run must reproduce the single-process oracle's pivot sequence and
every tableau bit.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import simplex_oracle as O


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, kind, m, n, seed, rule, q, K=0):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle.sharded_oracle import sharded_solve, sharded_windowed_solve
        from simplex_amd import dist as sdist, synth

        # 1. unique-id exchange (rank 0's id reaches everyone)
        uid = sdist.exchange_unique_id(make_id=lambda: bytes([7] * 100 + [rank] * 28))
        assert uid == bytes([7] * 100 + [0] * 28)
        # 2. this rank's row block, generated locally
        r0, r1 = sdist.row_partition(m, world, rank)
        T, obj, basis = synth.tableau_rows(kind, m, n, seed, r0, r1, order="C")
        T = np.array(T)

        def allgather(a):
            t = torch.from_numpy(a.astype(np.float64))
            out = [torch.empty_like(t) for _ in range(world)]
            dist.all_gather(out, t)
            return [o.numpy() for o in out]

        if K:
            st, hist = sharded_windowed_solve(T, obj, basis, r0, allgather, K=K, rule=rule,
                                              max_iters=5000)
        else:
            st, hist = sharded_solve(T, obj, basis, r0, allgather, rule=rule, max_iters=5000)
        q.put((rank, r0, r1, st, hist, T, obj, basis))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,kind,m,n,rule,K", [
    (2, "dense", 40, 56, "dantzig", 0),
    (3, "dense", 31, 45, "dantzig", 0),
    (2, "degenerate", 24, 24, "bland", 0),
    # the windowed protocol (the bench's N > 1 path): lazy column / row
    # reconstruction, one all-gather per pivot, a flush every K pivots
    (2, "dense", 40, 56, "dantzig", 4),
    (3, "dense", 31, 45, "dantzig", 8),
    (2, "degenerate", 24, 24, "bland", 8),
])
def test_sharded_protocol_matches_single_process(world, kind, m, n, rule, K):
    from simplex_amd import synth
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, kind, m, n, 3, rule, q, K))
             for r in range(world)]
    for p in procs:
        p.start()
    outs = sorted([q.get(timeout=120) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    T, basis = synth.full_tableau(kind, m, n, 3)
    st, hist = O.solve_tableau(T, basis, rule=rule, max_iters=5000)
    for rank, r0, r1, st_r, hist_r, T_r, obj_r, basis_r in outs:
        assert st_r == st and hist_r == hist
        assert np.array_equal(T_r, T[r0:r1])
        assert np.array_equal(obj_r, T[-1])
        assert np.array_equal(basis_r, basis)


def test_row_partition_covers_rows():
    from simplex_amd.dist import row_partition
    for m in (0, 1, 7, 8192, 8193):
        for w in (1, 2, 3, 8):
            blocks = [row_partition(m, w, r) for r in range(w)]
            assert blocks[0][0] == 0 and blocks[-1][1] == m
            assert all(a[1] == b[0] for a, b in zip(blocks, blocks[1:]))
            sizes = [b - a for a, b in blocks]
            assert max(sizes) - min(sizes) <= 1
