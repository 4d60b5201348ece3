"""Benchmark: pivots/s of the dense fp64 tableau simplex on MI355X.

Workload: BASELINE.json config 3, an 8192 x 16384 dense random-feasible LP,
tableau 8193 x 16385 fp64 (1.07 GB) resident in HBM before timing starts.

A "step" is one streaming pass of the hot path over the tableau: one window of
K pivots (K = 24 by default: K entering scans + ratio tests + pivot-row
normalisations, then ONE Gauss-Jordan elimination pass that applies all K
pivots).  With --window 0 a step is one single-pivot pass.  So
`--steps 20` times 20 x 24 = 480 pivots; `value` is pivots per second and
`ms_per_step` the time of one pass (K pivots).  With --gpus N > 1 (launched by
torch.distributed.run, one process per GPU) the SAME tableau is row-sharded
across the N GPUs (config 4): strong scaling, value = whole-job pivots/s.

Output: ONE JSON line on rank 0 (contract in the task statement), with
`roofline` for the elimination kernel (HIP-event timed inside the timed
region; algorithmic bytes = 16 B per touched tableau element)
and `cpu_baseline` (rank 0 at N=1 only): the C/OpenMP restatement of the
oracle (oracle/spx_oracle.c) on a bounded sample of the same workload with
this job's CPU share (OMP_NUM_THREADS threads), beside the same C code on 1
thread and the numpy oracle on 1 thread; every sample's pivots must equal the
GPU's.  `cpu_baseline.highs`: the reference's own engine (scipy linprog
'highs-ds', HiGHS) on config 2 beside the GPU's solve of the same LP; the
host load average is recorded beside every CPU figure.

At N > 1 the row-sharded persistent chain first passes a self-test on a small
LP (both leaving-row transports, pull and owner-push, byte-identical to the
reference path), then --peer-row auto times --row-trial windows of each on the
bench's own tableau and every rank takes the faster (config.peer_chain).
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "simplex-solver_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

METRIC = "pivots/sec + row-elim HBM GB/s (% roofline), fp64 dense tableau, 1/2/4/8 GPU"
DEFAULT_WINDOW = 24  # windowed elimination on one GPU (K sweep in profiles/r01)
HBM_PEAK_GBPS = 8000.0  # MI355X spec HBM3E peak (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # steps / warmup count tableau passes: windows of K pivots (1 pivot at --window 0)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--m", type=int, default=8192)
    ap.add_argument("--n", type=int, default=8192)
    ap.add_argument("--seed", type=int, default=20251205)
    ap.add_argument("--rule", default="dantzig")
    ap.add_argument("--dense", action="store_true", help="dense sweep (no zero-column skip)")
    ap.add_argument("--nt", type=int, default=-1,
                    help="elim non-temporal flags: 1 loads, 2 stores (-1: engine default)")
    ap.add_argument("--ilv", type=int, default=-1, help="elim interleaved columns (-1: default)")
    ap.add_argument("--R", type=int, default=0, help="elim rows per thread (0: auto)")
    ap.add_argument("--wgs", type=int, default=0, help="elim grid target (0: auto)")
    ap.add_argument("--fmap", type=int, default=-1,
                    help="windowed flush block map: 0 group-major (default), 1 chunk-major, "
                         "2 groups rotated by row chunk, 3 both; -1 default")
    ap.add_argument("--graph", type=int, default=1,
                    help="1: the timed region replays one hipGraph with an event pair "
                         "captured around every elimination; 0: direct launches + events")
    ap.add_argument("--ld-pad", type=int, default=-1, help="column padding (doubles)")
    ap.add_argument("--window", type=int, default=-1,
                    help="windowed elimination: K pivots per tableau pass (0 = off, "
                         "-1 = default: %d, on one GPU and on row shards)" % DEFAULT_WINDOW)
    ap.add_argument("--chain", type=int, default=0,
                    help="window pivot chain: 0 one persistent launch per window (default), "
                         "1 two launches per pivot, 2 / 3 persistent with 256- / 512-thread "
                         "blocks (at N > 1: the row-sharded chain's block width)")
    ap.add_argument("--chain-blocks", type=int, default=0, help="persistent chain grid (0: minimum)")
    ap.add_argument("--peer", type=int, default=1,
                    help="N > 1 windows: 1 the row-sharded persistent chain (peer records over "
                         "xGMI, after a bit-exact self-test against the RCCL path), 0 one RCCL "
                         "all-gather per pivot")
    ap.add_argument("--peer-row", default="auto", choices=["auto", "pull", "push"],
                    help="N > 1 peer chain: the leaving row's transport; auto times a few "
                         "windows of each after the self-test and every rank takes the faster")
    ap.add_argument("--row-trial", type=int, default=3,
                    help="windows per transport in the --peer-row auto trial")
    ap.add_argument("--same-device", action="store_true",
                    help="N > 1 rehearsal on ONE GPU: every rank on GPU 0, peer-only shards "
                         "(no RCCL, IPC-mapped peers), the self-test against the single-GPU "
                         "path; exercises the whole N > 1 bench path before an 8-GPU node")
    ap.add_argument("--time-every", type=int, default=0,
                    help="HIP events around every k-th elimination (or window flush) of the "
                         "timed region (0: every 8th elimination / flush; an event node costs "
                         "~6 us of stream time, and a timed window is launched directly: "
                         "~21 us per timed window at config 3)")
    ap.add_argument("--dump-history", default="",
                    help="diagnostic: rank 0 saves the run's pivot sequence (.npy) here")
    ap.add_argument("--cpu-seconds", type=float, default=15.0,
                    help="budget of the CPU-baseline sample (0 disables)")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles",
                                                           "traffic_r06.json"))
    return ap.parse_args()


def dist_env():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    return world, rank, local


def cpu_baseline(m, n, seed, rule, budget_s, gpu_hist):
    """Time the CPU oracle on the same config-3 tableau (rank 0, N=1 only).

    Primary figure: the C/OpenMP restatement (oracle/spx_oracle.c: p[j] == 0
    columns neither read nor written, touched columns as vectorised runs, rows
    over threads) with as many threads as this job's CPU share allows
    (OMP_NUM_THREADS, 16 per GPU on the box; the box's other cores belong to
    other jobs).  Also reported: the same C code on 1 thread and the numpy
    oracle (1 thread).  All must reproduce the GPU's first pivots exactly."""
    from oracle import c_oracle as C
    from oracle import simplex_oracle as O
    from simplex_amd import synth
    Tf, obj, basis0 = synth.tableau_rows("dense", m, n, seed, order="C")
    T = np.vstack([Tf, obj[None, :]])
    del Tf

    def c_run(threads, secs, Tc, bc, hist):
        C.set_threads(threads)
        k, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < secs and k < 5000:
            st, h = C.solve(Tc, bc, rule=rule, max_iters=1, hist_cap=1)
            if st != 1:  # no pivot made (optimal / unbounded)
                break
            hist += h
            k += 1
        return k, time.perf_counter() - t0

    def matches(h):
        kk = min(len(h), len(gpu_hist))
        return [tuple(x) for x in gpu_hist[:kk]] == h[:kk]

    threads = C.threads()  # OMP_NUM_THREADS
    Tc, bc, hist = T.copy(), basis0.copy(), []
    la0 = _loadavg()
    k, el = c_run(threads, budget_s * 0.6, Tc, bc, hist)
    la1 = _loadavg()
    # 1 thread, continuing the same sequence
    k1, el1 = c_run(1, budget_s * 0.2, Tc, bc, hist)
    la2 = _loadavg()
    # the thread-scaling curve between them (short samples, same sequence)
    scaling = {"1": k1 / el1 if el1 > 0 else None, str(threads): k / el}
    for tt in (2, 4, 8):
        if tt < threads:
            kt, elt = c_run(tt, budget_s * 0.06, Tc, bc, hist)
            scaling[str(tt)] = kt / elt if elt > 0 and kt else None
    C.set_threads(threads)
    del Tc
    ok = matches(hist)
    # numpy, 1 thread
    k2, hist2, t0 = 0, [], time.perf_counter()
    while time.perf_counter() - t0 < budget_s * 0.2 and k2 < 2000:
        c = O.select_entering(T[-1], T.shape[1] - 1, rule, 1e-9)
        r = O.ratio_test(T, c, basis0, rule, 1e-12)
        O.pivot(T, r, c)
        basis0[r] = c
        hist2.append((r, c))
        k2 += 1
    el2 = time.perf_counter() - t0
    ok2 = matches(hist2)
    la3 = _loadavg()
    host = _host_cpus()
    return {"value": k / el, "unit": "pivots/s", "cores": threads, "kind": "port",
            "sample": f"C/OpenMP oracle (oracle/spx_oracle.c), first {k} {rule} pivots of the "
                      f"same {m}x{n} tableau from the slack basis, {el:.1f} s, {threads} threads "
                      f"(this job's CPU share)",
            # host load (1/5/15-min os.getloadavg) before and after each sample:
            # the box's other jobs share its cores, and the figures move with them
            "loadavg": {"before": la0, "after": la1},
            "pivot_sequence_matches_gpu": bool(ok and ok2),
            "c_1thread": {"value": k1 / el1 if el1 > 0 else None, "pivots": k1,
                          "seconds": el1, "loadavg": {"before": la1, "after": la2}},
            "numpy_1thread": {"value": k2 / el2, "pivots": k2, "seconds": el2,
                              "matches_gpu": bool(ok2), "loadavg": {"before": la2, "after": la3}},
            "all_cores": _all_cores_projection(k / el, threads, host, alg_bytes_per_pivot(m, n),
                                               scaling),
            "host": host}


def _loadavg():
    try:
        return [round(x, 2) for x in os.getloadavg()]
    except OSError:
        return None


# BASELINE.json config 2 (seed 20251205 + its index, as tools/bench_configs.py)
CONFIG2 = (1024, 2048, 20251207)


def highs_beside(window):
    """The reference's real answer engine beside the GPU, on config 2 (rank 0,
    N = 1, after the timed region): scipy linprog(method='highs-ds') called as
    /root/reference/app/controllers/solver_controller.py:76-85 calls it (max
    -> negated c, A_ub / b_ub, bounds (0, None), presolve on) with the 10 s
    time_limit lifted, against this build's GPU engine solving the same LP to
    optimality through the C-ABI (K-pivot windows, the tableau loaded before
    the clock starts, as `value`).  Wall times, pivots / iterations, the two
    objectives and the host load."""
    from scipy.optimize import linprog
    from simplex_amd import synth
    from simplex_amd.engine import DeviceTableau
    m, n, seed = CONFIG2
    T, basis = synth.full_tableau("dense", m, n, seed)
    with DeviceTableau(0) as e:
        e.set_window(window)
        e.load(T, basis)
        e.solve(max_iters=5)  # warm: graph build, first launches
        e.load(T, basis)
        t0 = time.perf_counter()
        res = e.solve()
        gpu_s = time.perf_counter() - t0
    A, b, c = synth.lp_data("dense", m, n, seed)
    la0 = _loadavg()
    t0 = time.perf_counter()
    h = linprog(-c, A_ub=A, b_ub=b, bounds=[(0, None)] * n, method="highs-ds",
                options={"presolve": True})
    highs_s = time.perf_counter() - t0
    z = -h.fun
    return {"what": "scipy linprog(method='highs-ds') (HiGHS dual simplex, the reference's "
                    "answer path, solver_controller.py:76-85; time_limit lifted) on config 2 "
                    "vs this build's GPU solve of the same LP to optimality",
            "lp": f"config 2: {m}x{n} dense random-feasible LP (seed {seed})",
            "highs_seconds": highs_s, "highs_nit": int(h.nit), "highs_objective": z,
            "highs_status": int(h.status), "gpu_seconds": gpu_s, "gpu_pivots": int(res.iters),
            "gpu_objective": res.objective, "gpu_window": window,
            "objective_rel_diff": abs(res.objective - z) / abs(z),
            "gpu_speedup_wall": highs_s / gpu_s if gpu_s > 0 else None,
            "cores": 1, "loadavg": {"before": la0, "after": _loadavg()}}


# The pivot chain's latency floor per pivot (MI355X_MICROARCH.md price list,
# idle chip): an in-launch all-gather of a few KB among 32-256 CUs, and one
# dependent HBM miss.
CHAIN_EXCHANGE_FLOOR_US = 2.4
HBM_MISS_FLOOR_US = 0.4

# Host DRAM peak by CPU model (spec): EPYC 9005 "Turin" sockets have 12 DDR5-6400
# channels = 614.4 GB/s each.
HOST_DRAM_PEAK = {"EPYC 9575F": 614.4}


def alg_bytes_per_pivot(m, n):
    """Bytes one pivot must move on config 3 from the slack basis: read and
    write every element of the n + 1 touched columns."""
    return 16.0 * m * (n + 1)


def _all_cores_projection(v, threads, host, bytes_per_pivot, scaling=None):
    """The C oracle on every physical core is NOT run: the harness gives this
    job 16 threads (OMP_NUM_THREADS=16 on the box, the other cores belong to
    other jobs).  What is reported instead: the measured thread-scaling curve
    (1 .. `threads`), the rate scaled linearly to all physical cores, the
    rate extrapolated at the last measured doubling's efficiency, and the
    host's DRAM roofline (sockets x spec bandwidth / bytes per pivot) -- the
    CPU path is as memory-bound as the GPU's.  upper_bound = min(linear,
    roofline); estimate = min(doubling extrapolation, roofline)."""
    phys = host.get("physical_cores")
    model = host.get("model") or ""
    per_socket = next((bw for k, bw in HOST_DRAM_PEAK.items() if k in model), None)
    peak = per_socket * host["sockets"] if (per_socket and host.get("sockets")) else None
    lin = v * phys / threads if phys and threads else None
    roof = peak * 1e9 / bytes_per_pivot if peak else None
    cands = [x for x in (lin, roof) if x]
    est = None
    half = (scaling or {}).get(str(threads // 2))
    if phys and threads and half and v > half and phys > threads:
        import math
        est = v * (v / half) ** math.log2(phys / threads)  # each further doubling at that gain
        est = min(est, roof) if roof else est
    return {"measured": False,
            "why": "the harness caps this job at 16 host threads (OMP_NUM_THREADS=16)",
            "physical_cores": phys, "measured_scaling": scaling,
            "linear_projection": lin, "doubling_extrapolation": est,
            "host_dram_peak_GBps": peak, "dram_roofline_pivots_per_s": roof,
            "upper_bound": min(cands) if cands else None}


def _host_cpus():
    """Logical CPUs, sockets and physical cores of the host, this process's
    CPU affinity and OMP_NUM_THREADS (/proc/cpuinfo, sched_getaffinity)."""
    model, phys = None, set()
    pid = cid = None
    try:
        for line in open("/proc/cpuinfo"):
            k, _, v = line.partition(":")
            k, v = k.strip(), v.strip()
            if k == "model name" and model is None:
                model = v
            elif k == "physical id":
                pid = v
            elif k == "core id":
                cid = v
            elif not k and pid is not None:
                phys.add((pid, cid))
                pid = cid = None
        if pid is not None:
            phys.add((pid, cid))
    except OSError:
        pass
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = None
    return {"model": model, "logical_cpus": os.cpu_count(),
            "sockets": len({p for p, _ in phys}) or None, "physical_cores": len(phys) or None,
            "affinity_cpus": aff, "OMP_NUM_THREADS": os.environ.get("OMP_NUM_THREADS")}


def peer_selftest(eng, world, rank, K, tdist, torch, same_device=False, chain=0):
    """Before the timed run: the row-sharded persistent chain must reproduce the
    RCCL launch-per-phase path byte for byte on a small LP (every rank, all
    ranks agree), else the bench falls back to RCCL.  --same-device (peer-only
    shards, no RCCL): the reference is the single-GPU windowed path on the
    whole LP, and a failure ends the bench.  Both leaving-row transports run
    (pull, then owner-push) and must give the same bytes.  Returns (ok, note,
    push_ok)."""
    from simplex_amd import synth
    from simplex_amd.dist import row_partition
    from simplex_amd.engine import DeviceTableau, SpxError

    def all_ok(flag):
        t = torch.tensor([1 if flag else 0], dtype=torch.int64)
        tdist.all_reduce(t, op=tdist.ReduceOp.MIN)
        return bool(t.item())

    ms, ns = 256 * world, 2048
    r0, r1 = row_partition(ms, world, rank)
    T, obj, basis = synth.tableau_rows("dense", ms, ns, 99, r0, r1, order="F")
    kw = dict(max_iters=4 * K + 5)

    def run_peer(push):
        eng.set_chain(chain)
        eng.load_rows(T, obj, basis, ms, r0)
        eng.enable_peer_chain(push=push)
        if eng.chain_blocks() <= 0:
            return None
        eng.solve(**kw)
        return eng.history().tobytes(), eng.tableau().tobytes()

    note = "ok"
    try:
        a = run_peer(False)
        ok = a is not None
    except (SpxError, RuntimeError) as ex:
        ok, note = False, f"peer chain failed: {ex}"
    if not all_ok(ok):  # (every rank leaves here together: no collective is left pending)
        return False, note if not ok else "peer chain failed on another rank", False
    try:
        push_same = run_peer(True) == a
    except (SpxError, RuntimeError):
        push_same = False
    push_ok = all_ok(push_same)
    if same_device:
        Tw, objw, bw = synth.tableau_rows("dense", ms, ns, 99, 0, ms, order="F")
        with DeviceTableau(0) as ref:
            ref.set_window(K)
            ref.load_rows(Tw, objw, bw, ms, 0)
            ref.solve(**kw)
            full = ref.tableau()
            hist = ref.history()
        mine = np.vstack([full[r0:r1], full[-1:]])
        same = (hist.tobytes(), mine.tobytes()) == a
        ok = all_ok(same)
        return ok, ("ok (vs the single-GPU path)" if ok else
                    "peer chain differs from the single-GPU path"), push_ok and ok
    eng.set_chain(1)  # the RCCL all-gather path on the same LP
    eng.load_rows(T, obj, basis, ms, r0)
    eng.solve(**kw)
    same = (eng.history().tobytes(), eng.tableau().tobytes()) == a
    eng.set_chain(chain)
    ok = all_ok(same)
    return ok, "ok" if ok else "peer chain differs from the RCCL path: disabled", push_ok and ok


def select_row_transport(eng, K, opts, windows, world, tdist, torch, push_ok, rounds=2):
    """Time `windows` windows with each leaving-row transport, alternating
    pull / push for `rounds` rounds after the bench's warmup (the same pivots
    either way; they continue the run), max over ranks per trial and the
    fastest trial per transport, and let every rank take the same choice
    (dist.choose_row_transport).  Returns (choice, per-transport best ms per
    window, pivots made)."""
    from simplex_amd.dist import choose_row_transport
    ms, made = {}, 0
    modes = ("pull", "push") if push_ok else ("pull",)
    for _ in range(rounds):
        for mode in modes:
            eng.enable_peer_chain(push=(mode == "push"))
            tdist.barrier()
            eng.sync()
            t0 = time.perf_counter()
            eng.run_pivots(windows * K, **opts)
            eng.sync()
            t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
            tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
            ms[mode] = min(ms.get(mode, float("inf")), 1e3 * float(t.item()) / windows)
            made += windows * K
    return choose_row_transport(ms["pull"], ms.get("push"), push_ok), ms, made


def main():
    args = parse()
    world, rank, local = dist_env()
    if args.gpus != world and world > 1:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE {world}")
    use_graph = bool(args.graph)

    import torch  # device discovery / distributed plumbing only
    import torch.distributed as tdist
    from simplex_amd import synth
    from simplex_amd.dist import ShardedTableau, exchange_unique_id, row_partition
    from simplex_amd.engine import DeviceTableau

    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs a GPU (HIP); none visible")
    m, n = args.m, args.n
    if args.same_device and world < 2:
        raise SystemExit("--same-device needs WORLD_SIZE >= 2 (torch.distributed.run)")
    if world > 1 and args.same_device:
        # rehearsal of the N > 1 path on one GPU: no RCCL (it refuses two ranks
        # on one device), the peers IPC-mapped
        tdist.init_process_group("gloo")
        eng = ShardedTableau(0, rank, world, None, local="peer")
    elif world > 1:
        tdist.init_process_group("gloo")
        uid = exchange_unique_id()
        eng = ShardedTableau(local, rank, world, uid)
    else:
        eng = DeviceTableau(0)
    if args.ld_pad >= 0:
        eng.set_ld_pad(args.ld_pad)
    row0, row1 = row_partition(m, world, rank)
    Tf, obj, basis = synth.tableau_rows("dense", m, n, args.seed, row0, row1, order="F")
    K = args.window if args.window >= 0 else DEFAULT_WINDOW
    K = 0 if K <= 1 else K
    if K:
        eng.set_window(K)
    peer = None
    if args.same_device and not (K and args.peer):
        raise SystemExit("--same-device runs the peer chain only (--window > 1, --peer 1)")
    push_ok = False
    if world > 1 and K and args.peer:
        ok, note, push_ok = peer_selftest(eng, world, rank, K, tdist, torch, args.same_device,
                                          args.chain)
        peer = {"enabled": ok, "selftest": note, "push_selftest": push_ok}
        if args.same_device and not ok:
            raise SystemExit(f"--same-device: {note}")
    if world == 1 or (peer is not None and peer["enabled"]):
        # (at N > 1: the row-sharded chain's block width, modes 0 / 2 / 3)
        eng.set_chain(args.chain, args.chain_blocks)
    else:
        eng.set_chain(1)  # one RCCL all-gather per pivot
    eng.load_rows(Tf, obj, basis, m, row0)
    del Tf
    if peer is not None and peer["enabled"]:
        eng.enable_peer_chain(push=(args.peer_row == "push" and push_ok))
        if eng.chain_blocks() <= 0:
            raise SystemExit("row-sharded persistent chain passed its self-test but does not fit")
    if args.nt >= 0 or args.ilv >= 0 or args.R or args.wgs or args.fmap >= 0:
        fmap = max(args.fmap, 0) & 3
        if args.ilv >= 0:
            eng.set_elim_variant(args.R, args.wgs, -1 if args.nt < 0 else args.nt,
                                 args.ilv | fmap << 11)
        else:
            eng.set_elim_variant(args.R, args.wgs, -1 if args.nt < 0 else args.nt,
                                 flush_map=fmap)
    opts = dict(rule=args.rule, skip_zero_cols=not args.dense, use_graph=use_graph, chunk=32)

    def barrier():
        if world > 1:
            tdist.barrier()

    per_step = K if K else 1  # pivots per step (one tableau pass)
    n_warm, n_timed = args.warmup * per_step, args.steps * per_step
    # ranks start their first window together: a shard chain waits at most
    # 100 ms at its start handshake for the other ranks' blocks
    barrier()
    eng.run_pivots(n_warm, **opts)
    eng.sync()
    n_trial = 0
    if peer is not None and peer["enabled"]:
        if args.peer_row == "auto":
            # after the warmup: a few windows with each transport, alternating
            # (they count as warmup too), then every rank takes the faster one
            # (the same, from all-reduced times)
            choice, trial, n_trial = select_row_transport(eng, K, opts, args.row_trial, world,
                                                          tdist, torch, push_ok)
            peer["row_trial_ms_per_window"] = trial
        else:
            choice = "push" if (args.peer_row == "push" and push_ok) else "pull"
        eng.enable_peer_chain(push=(choice == "push"))
        peer["row_transport"] = choice
        # the re-import dropped the cached window graphs: rebuild them here,
        # outside the timed region, with one more window
        barrier()
        eng.run_pivots(per_step, **opts)
        eng.sync()
        n_trial += per_step
    eng.elim_timing(reset=True)
    barrier()
    eng.sync()
    t0 = time.perf_counter()
    every = args.time_every if args.time_every > 0 else 8
    eng.run_pivots(n_timed, time_elim=every, **opts)
    eng.sync()
    t1 = time.perf_counter()
    barrier()
    elapsed = t1 - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
        elapsed = float(t.item())
    status, iters, z = eng.state()
    if status != 4 or iters != n_trial + n_warm + n_timed:
        raise SystemExit(f"pivot loop ended early: status {status}, iters {iters}")
    ms_tot, launches, touched = eng.elim_timing(reset=True)
    chain = None
    if K and (world == 1 or (peer and peer["enabled"])):
        # the pivot chain, the other half of a window: HIP events around each
        # window's chain in 8 windows AFTER the timed region (event nodes cost
        # stream time, so they stay out of `value`)
        eng.set_chain_timing(True)
        eng.run_pivots(8 * K, **opts)
        eng.sync()
        c_ms, c_n = eng.chain_timing(reset=True)
        eng.set_chain_timing(False)
        nb = eng.chain_blocks()
        chain = {"kernel": ("spx::chain_shard_kernel" if world > 1 else "spx::chain_kernel")
                 if nb else "spx::lazy_ratio_kernel + spx::lazy_norm_kernel",
                 "bound": "latency: two in-launch all-to-all exchanges and two dependent "
                          "HBM gathers per pivot (DESIGN.md 4b)",
                 "blocks": nb, "avg_launch_us": 1e3 * c_ms / max(c_n, 1),
                 "us_per_pivot": 1e3 * c_ms / max(c_n * K, 1),
                 "share_of_step": (c_ms / max(c_n, 1)) / (1e3 * elapsed / args.steps),
                 "window": f"HIP events around the chain of {c_n} windows run after the "
                           f"timed region"}
        if nb:
            # the chain's latency roofline: per pivot two in-launch
            # all-to-all exchanges among the blocks and two dependent HBM gathers,
            # at MI355X_MICROARCH.md's idle-chip prices (all-gather among 32-256
            # CUs >= 2.4 us, a dependent HBM miss >= 0.4 us)
            floor = 2 * CHAIN_EXCHANGE_FLOOR_US + 2 * HBM_MISS_FLOOR_US
            chain["latency_floor_us_per_pivot"] = floor
            chain["frac_of_floor"] = floor / chain["us_per_pivot"] if chain["us_per_pivot"] else None
    what = "flush (window pass)" if K else "elimination"
    between = every - 1
    every = f"every {every}th"
    window = (f"timed region: HIP events on the engine stream around {every} {what}, "
              f"launched directly" + (" (the flush's start / stop events ride in its own launch, "
                                      "hipExtLaunchKernel: its dispatch span, as rocprofv3 "
                                      "measures it)" if K else "") + ("; of the windows in between, runs of 4 replay one "
                                      "hipGraph (SPX_GRAPH_WINDOWS), the rest are launched "
                                      "directly" if (use_graph and K and between) else ""))
    avg_ms = ms_tot / launches
    m_local = row1 - row0
    N = n + m + 1
    if K:
        # one flush per window; touched_total counts each flush's column list
        flushes = args.steps
        cols_per_launch = touched / flushes
        k_eff = K
        # read+write 16 B per listed element, plus the window's pivot columns
        # f_s (m) and pivot-row values p_s (listed columns)
        alg_bytes = 16.0 * m_local * cols_per_launch + 8.0 * k_eff * (m_local + cols_per_launch)
    else:
        cols_per_launch = touched / n_timed  # touched_total counts every pivot
        # algorithmic HBM bytes of one elimination launch: read+write 16 B for every
        # touched element except the entering column, which is only written (8 B)
        alg_bytes = 16.0 * m_local * (cols_per_launch - 1.0) + 8.0 * m_local
    dense_bytes = 16.0 * (m_local + 1) * N  # SURVEY §8(d) per-pivot figure (no skip)
    achieved = alg_bytes / (avg_ms * 1e-3) / 1e9
    traffic = None
    try:
        tj = json.load(open(args.traffic_json))
        key = f"{m}x{n}_w{world}_{'dense' if args.dense else 'skip'}" + (f"_k{K}" if K else "")
        traffic = tj.get(key, {}).get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        pass

    hist = eng.history() if rank == 0 else None
    if hist is not None and args.dump_history:
        np.save(args.dump_history, np.asarray(hist, dtype=np.int64))
    cpu = None
    if hist is not None and world == 1 and args.cpu_seconds > 0:
        cpu = cpu_baseline(m, n, args.seed, args.rule, args.cpu_seconds, hist.tolist())
        try:
            cpu["highs"] = highs_beside(K if K else 24)
        except Exception as ex:  # scipy missing or failed: say so, keep the line
            cpu["highs"] = {"error": f"{type(ex).__name__}: {ex}"}
    if rank == 0:
        value = n_timed / elapsed
        fvar = eng.elim_variant()
        kname = "spx::flush_lds_kernel" if K else "spx::elim_kernel"
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "pivots/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1e3 * elapsed / args.steps,
            "pivots_per_step": per_step,
            "pivots_timed": n_timed,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": f"synthetic: hash-seeded dense random-feasible LP (simplex_amd.synth, "
                    f"seed {args.seed})",
            "config": {"workload": ("config 3: 8192x16384 fp64 dense tableau" if world == 1
                                    else f"config 4: config-3 tableau row-sharded x{world}"
                                    + (" (rehearsal: every rank on GPU 0)" if args.same_device
                                       else "")),
                       "m": m, "n": n, "tableau": [m + 1, N], "rule": args.rule,
                       "elimination": "dense sweep" if args.dense else "skip p[j]==0 columns",
                       "timing": ("hipGraph replay (several windows per graph)"
                                  if (use_graph and K) else "direct launches"),
                       "elim_variant": fvar,
                       "step": (f"one tableau pass = a window of {K} pivots" if K
                                else "one pivot (single-pivot elimination pass)"),
                       "window": K,
                       "chain_blocks": eng.chain_blocks(),
                       "same_device": bool(args.same_device),
                       "parallelism": ("single GPU" if world == 1 else
                                       f"row-shard x{world}, " + (
                                           "one persistent chain launch per window, ratio "
                                           "records to every rank + the leaving row "
                                           + ("pushed by its owner into every peer's inbox"
                                              if peer.get("row_transport") == "push" else
                                              "gathered from its owner") + " (xGMI)"
                                           if peer and peer["enabled"] else
                                           "RCCL all-gather of [key | row] per pivot")),
                       "peer_chain": peer},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBPS,
                         "traffic": traffic,
                         "kernel": kname,
                         "avg_launch_us": avg_ms * 1e3,
                         "alg_bytes_per_launch": alg_bytes,
                         "touched_cols_per_launch": cols_per_launch,
                         "dense_equiv_GBps": dense_bytes / (avg_ms * 1e-3) / 1e9,
                         "window": window},
            "chain": chain,
            "cpu_baseline": cpu,
            "objective_after": z,
            # every pivot of the run (warmup, timed, chain timing) from the
            # slack basis: tests compare it with the oracle's fixture
            "pivots_total": int(len(hist)),
            "chain_reruns": int(eng.chain_reruns()) if hasattr(eng, "chain_reruns") else None,
            "pivots_sha256": hashlib.sha256(
                np.ascontiguousarray(hist, dtype="<i8").tobytes()).hexdigest(),
        }
        print(json.dumps(line), flush=True)
    eng.close()
    if world > 1:
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
