"""Multi-process RCCL check of the row-sharded pivot path.

Launch: python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \\
        tools/rccl_ranks_check.py [--m M --n N --pivots K --same-device]
Every rank loads its row block, runs the pivots through libspx's RCCL
all-gather, and rank 0 checks every rank's rows, the objective row and the
pivot sequence against the CPU oracle (bit-exact).  --same-device puts all ranks
on GPU 0 (only if the RCCL build allows several ranks per device).
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
    ap.add_argument("--m", type=int, default=300)
    ap.add_argument("--n", type=int, default=500)
    ap.add_argument("--pivots", type=int, default=0)
    ap.add_argument("--same-device", action="store_true")
    a = ap.parse_args()
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    local = int(os.environ.get("LOCAL_RANK", rank))
    from simplex_amd import dist as sdist, synth
    uid = sdist.exchange_unique_id()
    dev = 0 if a.same_device else local
    r0, r1 = sdist.row_partition(a.m, world, rank)
    T, obj, basis = synth.tableau_rows("dense", a.m, a.n, 17, r0, r1, order="F")
    with sdist.ShardedTableau(dev, rank, world, uid) as s:
        s.load_shard(T, obj, basis, a.m, r0)
        res = s.solve(max_iters=a.pivots, use_graph=True)
        out = (r0, r1, res.status, s.history().tolist(), s.tableau(), s.basis())
    outs = [None] * world
    dist.all_gather_object(outs, out)
    if rank == 0:
        from oracle import simplex_oracle as O
        Tf, bf = synth.full_tableau("dense", a.m, a.n, 17)
        st, hist = O.solve_tableau(Tf, bf, max_iters=a.pivots)
        ok = True
        for q, (r0, r1, stq, h, Tl, b) in enumerate(outs):
            good = ([tuple(x) for x in h] == hist and np.array_equal(Tl[:-1], Tf[r0:r1])
                    and np.array_equal(Tl[-1], Tf[-1]) and np.array_equal(b, bf))
            print(f"rank {q}: rows {r0}:{r1} status {stq} pivots {len(h)} bit-exact {good}")
            ok &= good
        print("RCCL_RANKS_CHECK", "PASS" if ok else "FAIL", f"world={world} pivots={len(hist)}")
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
