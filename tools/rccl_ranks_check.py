"""Multi-process check of the row-sharded pivot path.

Launch: python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \\
        tools/rccl_ranks_check.py [--rows M --cols N --pivots K --window K --peer P --same-device]
Every rank loads its row block and runs the pivots, then rank 0 checks every
rank's rows, the objective row and the pivot sequence against the CPU oracle
(bit-exact) and exits non-zero on a mismatch.

  --peer 0  RCCL all-gather per pivot (launch-per-phase windows, or single pivots)
  --peer 1  RCCL context + the row-sharded persistent chain (IPC-mapped peers)
  --peer 2  no communicator at all: the persistent chain's peers only
            (spx_create_sharded_peer; works with several ranks on one GPU,
            which RCCL refuses)
--same-device puts all ranks on GPU 0.  (--rows / --cols: torch.distributed.run
would take --m / --n as abbreviations of its own options.)
--then "R1xC1,R2xC2,...": after the first LP, reload the SAME context with
each of these LPs in turn (re-export / re-import of the peers, so a rank's
freed-and-reallocated buffers are mapped again), checking each run.
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "simplex-solver_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=300)
    ap.add_argument("--cols", type=int, default=500)
    ap.add_argument("--pivots", type=int, default=0)
    ap.add_argument("--window", type=int, default=0)
    ap.add_argument("--peer", type=int, default=0, choices=[0, 1, 2])
    ap.add_argument("--rule", default="dantzig")
    ap.add_argument("--kind", default="dense")
    ap.add_argument("--seed", type=int, default=17)
    ap.add_argument("--same-device", action="store_true")
    ap.add_argument("--then", default="", help="reload sizes, e.g. 200x2000,600x900")
    a = ap.parse_args()
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    local = int(os.environ.get("LOCAL_RANK", rank))
    from simplex_amd import dist as sdist, synth
    dev = 0 if a.same_device else local
    sizes = [(a.rows, a.cols)] + [tuple(int(x) for x in z.split("x"))
                                  for z in a.then.split(",") if z]
    if a.peer == 2:
        s = sdist.ShardedTableau(dev, rank, world, local="peer")
    else:
        s = sdist.ShardedTableau(dev, rank, world, sdist.exchange_unique_id())
    runs = []
    with s:
        s.set_window(a.window)
        for rows, cols in sizes:  # one context, reloaded for every LP
            r0, r1 = sdist.row_partition(rows, world, rank)
            T, obj, basis = synth.tableau_rows(a.kind, rows, cols, a.seed, r0, r1, order="F")
            s.load_shard(T, obj, basis, rows, r0)
            if a.peer:
                s.enable_peer_chain()
            blocks = s.chain_blocks()
            res = s.solve(max_iters=a.pivots, rule=a.rule, use_graph=True)
            out = (r0, r1, res.status, s.history().tolist(), s.tableau(), s.basis(), blocks)
            outs = [None] * world
            dist.all_gather_object(outs, out)
            runs.append(outs)
    ok = True
    if rank == 0:
        from oracle import simplex_oracle as O
        for (rows, cols), outs in zip(sizes, runs):
            Tf, bf = synth.full_tableau(a.kind, rows, cols, a.seed)
            st, hist = O.solve_tableau(Tf, bf, rule=a.rule, max_iters=a.pivots)
            for q, (r0, r1, stq, h, Tl, b, nb) in enumerate(outs):
                good = ([tuple(x) for x in h] == hist and np.array_equal(Tl[:-1], Tf[r0:r1])
                        and np.array_equal(Tl[-1], Tf[-1]) and np.array_equal(b, bf)
                        and stq == st)
                print(f"{rows}x{cols} rank {q}: rows {r0}:{r1} status {stq} pivots {len(h)} "
                      f"chain blocks {nb} bit-exact {good}", flush=True)
                ok &= good
            if a.peer:
                ok &= all(o[6] > 0 for o in outs)  # the persistent chain ran
        print("RCCL_RANKS_CHECK", "PASS" if ok else "FAIL",
              f"world={world} peer={a.peer} window={a.window} loads={len(sizes)}", flush=True)
    flag = [ok]
    dist.broadcast_object_list(flag, src=0)
    dist.destroy_process_group()
    sys.exit(0 if flag[0] else 1)


if __name__ == "__main__":
    main()
