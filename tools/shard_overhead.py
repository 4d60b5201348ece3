"""Per-pivot cost of the row-sharded path at the config-4 shard shape, on one
GPU.  Every rank holds SHARD_ROWS (1024) rows x all 16385
columns of the config-3 tableau; a rank's LP is rows [0, world * 1024) with its
own basis entries and the shared objective row.

  single        the single-GPU engine on one 1024-row block (N = 1 kernels)
  rccl1         1-rank RCCL communicator: prep -> all-gather -> finish per pivot
  peer1         1-rank row-sharded persistent chain (chain_shard_kernel)
  peer2v/peer3v 2 / 3 virtual ranks (threads, one stream each) of 1024 rows,
                the row-sharded persistent chain: ratio records to every rank,
                row gather from the owner's tableau (in-process peers)
  lazy2v        2 virtual ranks, launch-per-phase + in-process all-gather

Prints one JSON line per mode: microseconds per pivot over SHARD_PIVOTS pivots
after 20 warm-up pivots (windows of SHARD_WINDOWS, default 24).
"""
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "simplex-solver_amd"))

from simplex_amd import dist, synth  # noqa: E402
from simplex_amd.engine import DeviceTableau  # noqa: E402

m, n, rows = 8192, 8192, int(os.environ.get("SHARD_ROWS", "1024"))
K = int(os.environ.get("SHARD_WINDOWS", "24"))
k = int(os.environ.get("SHARD_PIVOTS", "480"))
MODES = os.environ.get("SHARD_MODES", "single,rccl1,peer1,peer2v,peer3v,lazy2v").split(",")


def one_rank(mode):
    T, obj, basis = synth.tableau_rows("dense", m, n, 20251205, 0, rows, order="F")
    if mode == "single":
        eng = DeviceTableau(0)
    elif mode == "rccl1":
        eng = dist.ShardedTableau(0, 0, 1, dist.make_unique_id())
    else:
        eng = dist.ShardedTableau(0, 0, 1, local="peer")
    with eng:
        eng.set_window(K)
        eng.load_rows(T, obj, basis[:rows], rows, 0)
        if mode == "peer1":
            eng.enable_peer_chain(allgather=lambda b: [b])
        eng.run_pivots(20)
        eng.sync()
        t0 = time.perf_counter()
        eng.run_pivots(k)
        eng.sync()
        el = time.perf_counter() - t0
        st, it, _ = eng.state()
        return el, st, it, eng.chain_blocks()


def virtual_ranks(world, peer):
    uid = bytes([world, 31, 7]) + os.urandom(125)
    bar = threading.Barrier(world)
    res, errs = {}, []

    def rank_main(rank):
        try:
            r0 = rank * rows
            T, obj, basis = synth.tableau_rows("dense", m, n, 20251205, r0, r0 + rows, order="F")
            with dist.ShardedTableau(0, rank, world, uid, local=True) as s:
                s.set_window(K)
                s.load_shard(T, obj, basis[:world * rows], world * rows, r0)
                if peer:
                    s.enable_peer_chain()
                s.run_pivots(20)
                s.sync()
                bar.wait()
                t0 = time.perf_counter()
                s.run_pivots(k)
                s.sync()
                el = time.perf_counter() - t0
                bar.wait()
                st, it, _ = s.state()
                res[rank] = (el, st, it, s.chain_blocks())
        except Exception as ex:  # noqa: BLE001
            errs.append(repr(ex))
            bar.abort()

    th = [threading.Thread(target=rank_main, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    if errs:
        raise RuntimeError(errs)
    el = max(v[0] for v in res.values())
    return el, res[0][1], res[0][2], res[0][3]


for mode in MODES:
    if mode in ("single", "rccl1", "peer1"):
        el, st, it, nb = one_rank(mode)
        world = 1
    else:
        world = int(mode[-2])
        el, st, it, nb = virtual_ranks(world, peer=mode.startswith("peer"))
    print(json.dumps({"mode": mode, "ranks": world, "window": K, "rows_per_rank": rows,
                      "cols": n + m + 1, "pivots": k, "us_per_pivot": 1e6 * el / k,
                      "pivots_per_s": k / el, "chain_blocks": nb, "status": st, "iters": it}),
          flush=True)
