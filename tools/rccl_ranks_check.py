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
--chain M: the persistent chain's mode (3: 512-thread blocks, so 8 ranks' 32
blocks fit one GPU's 256 CUs with --same-device).  --push: the owner-push row
transport (spx_set_peer_push).  --fixture NAME: check against the fullsize
fixture (tests/golden/fullsize.json: the oracle's pivot prefix and the
assembled tableau's SHA-256 checkpoint after --pivots) instead of running the
oracle here (config 3 is 1 GB).  --ipc-log: print every rank's exported
addresses, IPC handle digests and mapped peer pointers per load (DESIGN.md
§5c); --no-solve skips the pivots (the IPC diagnostic alone).
--fake-groups: every rank its own device group although all share GPU 0
(SPX_PEER_GROUP_TAG), so the start handshake runs the cross-group verdict
wait of ranks on different GPUs (keep all ranks' blocks within the CUs).
--run-pivots: enqueue the pivots with spx_run_pivots (no host wait) and drain
with spx_sync, instead of spx_solve; --late-drain S: the last rank sleeps S
seconds before its drain (a window aborted at its start handshake is rerun at
the drain points, which then happen S seconds apart: ADVICE r4, spx.h).
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
    ap.add_argument("--chain", type=int, default=0)
    ap.add_argument("--push", action="store_true")
    ap.add_argument("--fixture", default="")
    ap.add_argument("--ipc-log", action="store_true")
    ap.add_argument("--no-solve", action="store_true")
    ap.add_argument("--abort-every", type=int, default=0,
                    help="force a start-handshake abort of every k-th window (test hook)")
    ap.add_argument("--run-pivots", action="store_true")
    ap.add_argument("--late-drain", type=float, default=0.0)
    ap.add_argument("--fake-groups", action="store_true",
                    help="each rank its own device group (SPX_PEER_GROUP_TAG=rank): the "
                         "multi-GPU handshake's cross-group verdict wait on one GPU")
    ap.add_argument("--end-no-import", default="",
                    help="after the checked LPs, reload these sizes WITHOUT a peer import "
                         "(no pivots), check no exported buffer was freed, time the destroy")
    a = ap.parse_args()
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    local = int(os.environ.get("LOCAL_RANK", rank))
    if a.fake_groups:
        os.environ["SPX_PEER_GROUP_TAG"] = str(rank)
    from simplex_amd import dist as sdist, synth
    dev = 0 if a.same_device else local
    sizes = [(a.rows, a.cols)] + [tuple(int(x) for x in z.split("x"))
                                  for z in a.then.split(",") if z]
    if a.peer == 2:
        s = sdist.ShardedTableau(dev, rank, world, local="peer")
    else:
        s = sdist.ShardedTableau(dev, rank, world, sdist.exchange_unique_id())
    runs = []
    pool_ok = True
    import hashlib
    with s:
        s.set_window(a.window)
        s.set_chain(a.chain)
        if a.abort_every:
            s.set_chain_handshake(-a.abort_every)
        for rows, cols in sizes:  # one context, reloaded for every LP
            r0, r1 = sdist.row_partition(rows, world, rank)
            T, obj, basis = synth.tableau_rows(a.kind, rows, cols, a.seed, r0, r1, order="F")
            s.load_shard(T, obj, basis, rows, r0)
            del T
            blob_digest = None
            if a.peer:
                blobs = []

                def allgather(blob):
                    out = [None] * world
                    dist.all_gather_object(out, blob)
                    blobs.extend(out)
                    return out
                s.enable_peer_chain(allgather=allgather, push=a.push)
                # the IPC handles of every rank's tableau and record buffer
                blob_digest = [hashlib.sha256(b[16:144]).hexdigest()[:16] for b in blobs]
            if a.ipc_log:
                d = s.peer_debug() if a.peer else {}
                print(f"IPC {rows}x{cols} rank {rank}: A {d.get('A', 0):#x} records "
                      f"{d.get('records', 0):#x} gen {d.get('gen')} handles {blob_digest} "
                      f"mapped A {[hex(x) for x in d.get('peer_A', [])]} records "
                      f"{[hex(x) for x in d.get('peer_records', [])]}", flush=True)
            blocks = s.chain_blocks()
            if a.peer and blocks > 0 and rows == sizes[0][0]:
                g = s.peer_groups()
                print(f"rank {rank}: device groups {g['groups']} (this rank's: {g['group']}, "
                      f"{g['members']} member(s))", flush=True)
            if a.no_solve:
                runs.append(None)
                continue
            if a.run_pivots:
                import time
                from simplex_amd import _lib as L
                s.run_pivots(a.pivots, rule=a.rule, use_graph=True)
                if a.late_drain and rank == world - 1:
                    time.sleep(a.late_drain)
                t0 = time.perf_counter()
                s.sync()
                drain_s = time.perf_counter() - t0
                stq = s.state()[0]
                stq = 1 if stq == L.SPX_RUNNING else stq  # (the request's end = the oracle's limit)
                print(f"rank {rank}: drain {drain_s:.3f} s, chain reruns {s.chain_reruns()}",
                      flush=True)
            else:
                stq = s.solve(max_iters=a.pivots, rule=a.rule, use_graph=True).status
            Tl = s.tableau()
            out = (r0, r1, stq, s.history().tolist(), Tl if not a.fixture else None,
                   s.basis(), blocks, s.chain_reruns(), s.peer_push() if a.peer else -1)
            outs = [None] * world
            dist.all_gather_object(outs, out)
            parts = [None] * world if rank == 0 else None
            if a.fixture:  # the rows go to rank 0 only (1 GB at config 3)
                dist.gather_object(Tl, parts, dst=0)
            del Tl
            runs.append((outs, parts))
        # reloads whose buffers come back from the pool and are not
        # exported again must return them to the pool (never hipFree), and the
        # destroy then has no release marks to wait for in them
        for z in [z for z in a.end_no_import.split(",") if z]:
            rows, cols = (int(x) for x in z.split("x"))
            r0, r1 = sdist.row_partition(rows, world, rank)
            T, obj, basis = synth.tableau_rows(a.kind, rows, cols, a.seed, r0, r1, order="F")
            s.load_shard(T, obj, basis, rows, r0)
            d = s.peer_pool_debug()
            print(f"rank {rank}: reload {rows}x{cols} without import: exported {d['exported']} "
                  f"held {d['held']} pooled {d['pooled']}", flush=True)
            if d["held"] != d["exported"]:
                print(f"rank {rank}: an exported buffer was freed", flush=True)
                pool_ok = False
        if a.end_no_import:
            import time
            dist.barrier()
            t_close = time.perf_counter()
    if a.end_no_import:
        print(f"rank {rank}: destroy {time.perf_counter() - t_close:.3f} s", flush=True)
    ok = pool_ok
    if rank == 0 and not a.no_solve:
        from oracle import simplex_oracle as O
        for (rows, cols), (outs, parts) in zip(sizes, runs):
            print(f"{rows}x{cols}: chain reruns per rank {[o[7] for o in outs]}, row transport "
                  f"{['push' if o[8] == 1 else 'pull' if o[8] == 0 else '-' for o in outs]}",
                  flush=True)
            if a.fixture:
                import json
                gold = os.path.join(ROOT, "tests", "golden")
                fx = json.load(open(os.path.join(gold, "fullsize.json")))[a.fixture]
                hist = [tuple(x) for x in np.load(os.path.join(
                    gold, f"fullsize_{a.fixture}.npz"))["hist"][:a.pivots].tolist()]
                assert (fx["m"], fx["n"], fx["seed"]) == (rows, cols, a.seed), "fixture LP differs"
                Tall = np.vstack([p_[:-1] for p_ in parts] + [parts[0][-1:]])
                dig = hashlib.sha256(np.ascontiguousarray(Tall).tobytes()).hexdigest()
                good_t = dig == fx["checkpoint_sha256"][str(a.pivots)]
                same_obj = all(np.array_equal(p_[-1], parts[0][-1]) for p_ in parts)
                print(f"assembled tableau after {a.pivots} pivots: sha256 {dig[:16]} "
                      f"fixture match {good_t}, objective rows equal {same_obj}", flush=True)
                ok &= good_t and same_obj
                for q, (r0, r1, stq, h, _, b, nb, *_r) in enumerate(outs):
                    good = [tuple(x) for x in h] == hist and stq == 1
                    print(f"rank {q}: rows {r0}:{r1} status {stq} pivots {len(h)} chain blocks {nb} "
                          f"pivots = fixture {good}", flush=True)
                    ok &= good and np.array_equal(b, outs[0][5])
            else:
                Tf, bf = synth.full_tableau(a.kind, rows, cols, a.seed)
                st, hist = O.solve_tableau(Tf, bf, rule=a.rule, max_iters=a.pivots)
                for q, (r0, r1, stq, h, Tl, b, nb, *_r) in enumerate(outs):
                    good = ([tuple(x) for x in h] == hist and np.array_equal(Tl[:-1], Tf[r0:r1])
                            and np.array_equal(Tl[-1], Tf[-1]) and np.array_equal(b, bf)
                            and stq == st)
                    print(f"{rows}x{cols} rank {q}: rows {r0}:{r1} status {stq} pivots {len(h)} "
                          f"chain blocks {nb} bit-exact {good}", flush=True)
                    ok &= good
            if a.peer:
                ok &= all(o[6] > 0 for o in outs)  # the persistent chain ran
                ok &= all(o[8] == (1 if a.push else 0) for o in outs)
        print("RCCL_RANKS_CHECK", "PASS" if ok else "FAIL",
              f"world={world} peer={a.peer} window={a.window} loads={len(sizes)} "
              f"push={int(a.push)} chain={a.chain}", flush=True)
    flag = [ok]
    dist.broadcast_object_list(flag, src=0)
    dist.destroy_process_group()
    sys.exit(0 if flag[0] else 1)


if __name__ == "__main__":
    main()
