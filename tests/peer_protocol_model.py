"""Executable model of the row-sharded persistent chain's cross-rank protocol.

TEST INFRASTRUCTURE (imported by tests/test_peer_protocol_model.py only).

The CPU suite's other sharded test (test_dist_gloo.py) restates the RCCL
fallback: one all-gather per pivot, synchronous.  The default N > 1 protocol is
different and asynchronous (csrc/spx_chain.hpp, chain_shard_kernel and
chain_start): every rank's blocks run free, write their ratio
records into EVERY rank's buffer and poll only their own, and the ranks
interlock only through those records.  This module restates that protocol with
one Python thread per (rank, block), "device memory" as shared dicts of tagged
granules, and optional delays at the points where the GPU's timing varies, so
its hazards can be exercised on a CPU:

  * ratio records in two halves by pivot parity: a rank whose entering
    exchange is local may publish pivot q+1's ratio record before a slower
    peer has read pivot q's (never q+2);
  * the leaving row gathered from its OWNER's stale rows (a peer pointer), with
    the pending slots applied from the winning record's f history;
  * the window-end "done" barrier: no rank's flush rewrites its rows while a
    peer may still gather one of them;
  * rank 0's time-limit stop bit riding in its ratio records;
  * the start handshake: arrival granules, a verdict fixed once per window by
    compare-and-swap (GO / ABORT), the host's rerun of an aborted window;
  * the poll's geometry: wave 0 of a block reads the nr * B record headers as
    64 lanes x RPL records (RPL = 1, 2, 4, 8; clamped indices), which covers
    every slot only while nr * B <= CHAIN_SH_SLOTS = 512 (config 4: 8 ranks x
    64 blocks is exactly that);
  * device groups (round 6, `groups=`): ranks on different GPUs each settle
    their own group's arrivals and verdict, then wait for every other group's
    verdict; a group still undecided after the handshake bound is decided
    ABORT(W) by a compare-and-swap on its word (mutant `no_group_cas`: the
    round-5 wait, which runs into the spin bound when a group is late);
  * the owner-push row transport (round 5, `push=True`): the leaving row's
    owner writes its stale values into every peer's inbox (tagged granules, two
    halves by pivot parity) instead of every peer reading the owner's rows; the
    window-end barrier is then not needed, since no peer reads another rank's
    rows.

The arithmetic is the spec's operation for operation: Python
floats are IEEE doubles and `v - f * p` rounds the product, then the
difference, as the kernels (-ffp-contract=off) and the numpy oracle do.  So a
correct protocol reproduces the oracle bit for bit, and a broken one (the
`mutant` switches) shows up as a wrong tableau or a wait that never ends.
"""
from __future__ import annotations

import math
import threading
import time

import numpy as np

GO, ABORT = 1, 2
RATIO, ENTER, DONE, START = 0, 1, 2, 3


class Timeout(RuntimeError):
    """A bounded wait ran out (the model's ST_FAULT)."""


def _tag(W, q, kind):
    return (W, q, kind)


def apply_sel(v, i_is_r, j_is_c, f, p, skip=True):
    """One pending slot on one stale element (spx_delayed.hpp apply_sel)."""
    if j_is_c:
        return 1.0 if i_is_r else 0.0
    if skip and p == 0.0:
        return v
    if i_is_r:
        return p
    return v - f * p


CHAIN_SH_SLOTS = 512  # spx_chain.hpp: ratio record slots one poll covers


def poll_slots(BR):
    """The record slots wave 0 of a block reads in one poll pass
    (spx_chain.hpp poll_records_n): lane l reads l, l + 64, ... (RPL records
    per lane), clamped to BR - 1, so no lane branches around its loads."""
    if BR > CHAIN_SH_SLOTS:
        raise ValueError(f"{BR} ratio records exceed one poll ({CHAIN_SH_SLOTS})")
    rpl = 1 if BR <= 64 else 2 if BR <= 128 else 4 if BR <= 256 else 8
    return sorted({min(lane + 64 * x, BR - 1) for lane in range(64) for x in range(rpl)})


class Device:
    """What every rank can reach: its peers' record buffers and stale rows."""

    def __init__(self, nr, B, mutant=(), push=False, groups=None):
        self.nr, self.B, self.mutant, self.push = nr, B, set(mutant), push
        # device group of each rank (ranks sharing a GPU); one group by default
        self.group_of = list(groups) if groups is not None else [0] * nr
        self.ngroups = max(self.group_of) + 1
        self.verdicts = [(0, 0)] * self.ngroups
        halves = 1 if "one_half" in self.mutant else 2
        self.slots = poll_slots(nr * B)
        assert self.slots == list(range(nr * B)), "the poll misses a record slot"
        self.ratio = [[dict() for _ in range(halves)] for _ in range(nr)]
        # owner-push inboxes: [rank][parity half][column] -> (tag, stale value)
        self.inbox = [[dict() for _ in range(2)] for _ in range(nr)]
        self.enter = [dict() for _ in range(nr)]
        self.done = [dict() for _ in range(nr)]
        self.arrive = {}
        self.cas = threading.Lock()
        self.A = [None] * nr       # each rank's stale rows (read by peers' row gathers)
        self.row0 = [0] * nr

    def half(self, it0, q):
        return 0 if "one_half" in self.mutant else (it0 + q) & 1


WAIT_LIMIT = 5.0  # s: the model's bound on every spin (the kernels' ~4 s)
# Pause between polls.  0 yields the GIL at once; with hundreds of block
# threads (config 4's 8 x 64) the spinning threads would starve the working
# ones, so large worlds poll every POLL_SLEEP seconds instead.
POLL_SLEEP = 0.0


def _wait(pred, what, limit=None):
    limit = WAIT_LIMIT if limit is None else limit
    t0 = time.monotonic()
    while True:
        v = pred()
        if v is not None:
            return v
        if time.monotonic() - t0 > limit:
            raise Timeout(what)
        time.sleep(POLL_SLEEP)


def _wait_all(get, keys, ok, what, limit=None):
    """Poll until one pass sees ok(get(k)) for every key, and return that
    pass's values (as the kernels' polls do).  Slots seen matching are not
    re-read on every pass while the others are awaited -- only the final pass
    re-reads them all -- so a wait costs about one pass over the slots, not one
    per poll: with 512 polling block threads (config 4) the full re-read of
    every pass starved the threads that do the work."""
    keys = list(keys)
    nxt = 0

    def pred():
        nonlocal nxt
        while nxt < len(keys) and ok(get(keys[nxt])):
            nxt += 1
        if nxt < len(keys):
            return None
        vals = [get(k) for k in keys]
        for x, v in enumerate(vals):
            if not ok(v):
                nxt = x
                return None
        return vals
    return _wait(pred, what, limit)


def _argmin(keys):
    """Lexicographic winner of (value, tie, payload...) tuples (None: no key)."""
    keys = [k for k in keys if k is not None]
    return min(keys) if keys else None


class Rank:
    """One rank: its stale rows, replicated objective row / basis, and the
    host loop (windows, flush, reruns)."""

    def __init__(self, dev, rank, A_loc, obj, basis, row0, K, rule="dantzig",
                 eps_opt=1e-9, eps_piv=1e-12, delay=None, hs_bound=0.5, late=None):
        self.dev, self.rank = dev, rank
        self.A = np.array(A_loc, dtype=np.float64)
        self.obj = np.array(obj, dtype=np.float64)
        self.basis = np.array(basis, dtype=np.int64)
        self.row0, self.K, self.rule = row0, K, rule
        self.eps_opt, self.eps_piv = eps_opt, eps_piv
        self.m_local, self.N = self.A.shape
        self.hist = []
        self.status = 4            # SPX_RUNNING
        self.epoch = 0
        self.it = 0
        self.reruns = 0
        self.delay = delay or (lambda *a: None)
        self.hs_bound = hs_bound
        self.late = late or (lambda *a: 0.0)  # extra start delay of a block (W, b) -> s
        self.stop = threading.Event()
        dev.A[rank], dev.row0[rank] = self.A, row0

    # ---- the window: B block threads (one persistent launch) ----------------
    def window(self, npiv):
        dev, B, N, m_local = self.dev, self.dev.B, self.N, self.m_local
        W = self.epoch + 1
        it0 = self.it
        cpb = -(-(N - 1) // B)
        rpb = max(1, -(-m_local // B))
        stop0 = self.rank == 0 and self.stop.is_set()
        # pivot 0's entering column: the previous kernel's partials (kernel boundary)
        c0 = self._enter0()
        shared = dict(made=0, status=4, r=[], c=[], f={}, p={}, prhs=[], err=None, abort=False)
        obj_new = self.obj.copy()
        lock = threading.Lock()

        def block(b):
            try:
                self._block(b, W, it0, npiv, cpb, rpb, c0, stop0, shared, obj_new, lock)
            except Exception as ex:  # noqa: BLE001 - surfaced by the host loop
                shared["err"] = ex

        th = [threading.Thread(target=block, args=(b,)) for b in range(B)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        if shared["err"] is not None:
            raise shared["err"]
        if shared["abort"]:
            return "notres"
        self.epoch = W
        # flush + bookkeeping (the window's made slots, on this rank's rows)
        q = shared["made"]
        for s in range(q):
            self.hist.append((shared["r"][s], shared["c"][s]))
            self.basis[shared["r"][s]] = shared["c"][s]
        for i in range(m_local):
            ig = self.row0 + i
            for j in range(N):
                v = self.A[i, j]
                for s in range(q):
                    p = shared["p"][s][j] if j < N - 1 else shared["prhs"][s]
                    v = apply_sel(v, ig == shared["r"][s], j == shared["c"][s],
                                  shared["f"][s][i], p)
                self.A[i, j] = v
        self.obj = obj_new
        self.it += q
        if shared["status"] != 4:
            self.status = shared["status"]
        return "ok"

    def _enter0(self):
        o = self.obj[:self.N - 1]
        cand = [j for j in range(self.N - 1) if o[j] < -self.eps_opt]
        if not cand:
            return -1
        if self.rule == "bland":
            return cand[0]
        return min(cand, key=lambda j: (o[j], j))

    def _start(self, b, W):
        """chain_start: arrival granule, bounded wait for my device group, its
        verdict by compare-and-swap (first writer for window W wins), then --
        ranks on several GPUs -- every other group's verdict."""
        dev = self.dev
        g = dev.group_of[self.rank]
        slot = self.rank * dev.B + b
        time.sleep(self.late(W, b))
        dev.arrive[slot] = _tag(W, 0, START)
        t0 = time.monotonic()
        want = GO
        mine = [r * dev.B + x for r in range(dev.nr) if dev.group_of[r] == g
                for x in range(dev.B)]
        nxt, n = 0, len(mine)  # (arrivals seen are not re-read: see _wait_all)
        while True:
            while nxt < n and dev.arrive.get(mine[nxt]) == _tag(W, 0, START):
                nxt += 1
            if nxt == n and all(dev.arrive.get(x) == _tag(W, 0, START) for x in mine):
                break
            if dev.verdicts[g][0] >= W:
                break  # (the group's word already holds W: decided)
            if time.monotonic() - t0 > self.hs_bound:
                want = ABORT
                break
            time.sleep(POLL_SLEEP)
        with dev.cas:
            vw, vs = dev.verdicts[g]
            if vw > W:
                return ABORT  # the group is past W: W was aborted
            if vw < W:
                dev.verdicts[g] = (W, want)
                vs = want
        if vs != GO or dev.ngroups == 1:
            return vs
        # every other group's verdict; an undecided one is aborted by CAS once
        # the handshake bound has passed (round 6; spx_chain.hpp chain_start)
        t_end = time.monotonic() + WAIT_LIMIT
        while True:
            dec, ab = True, False
            for h in range(dev.ngroups):
                vw, vs = dev.verdicts[h]
                if (vw < W and "no_group_cas" not in dev.mutant
                        and time.monotonic() - t0 > self.hs_bound):
                    with dev.cas:
                        if dev.verdicts[h][0] < W:
                            dev.verdicts[h] = (W, ABORT)
                        vw, vs = dev.verdicts[h]
                dec &= vw >= W
                ab |= vw > W or (vw == W and vs == ABORT)
            if ab:
                return ABORT
            if dec:
                return GO
            if time.monotonic() > t_end:
                raise Timeout(f"rank {self.rank}: other groups' verdicts for window {W}")
            time.sleep(POLL_SLEEP)

    def _block(self, b, W, it0, npiv, cpb, rpb, c0, stop0, sh, obj_new, lock):
        dev, B, N, nr, rank = self.dev, self.dev.B, self.N, self.dev.nr, self.rank
        if self._start(b, W) != GO:
            with lock:
                sh["abort"] = True  # nothing stored: the host reruns the window
            return
        cols = list(range(b * cpb, min((b + 1) * cpb, N - 1)))
        rows = list(range(b * rpb, min((b + 1) * rpb, self.m_local)))
        o = {j: self.obj[j] for j in cols}
        bcur = {i: self.A[i, N - 1] for i in rows}
        bas = {i: self.basis[self.row0 + i] for i in rows}
        fh = {i: [] for i in rows}      # f_s[i] of my rows
        ph = {j: [] for j in cols}      # p_s[j] of my columns
        slots = []                       # (r_s, c_s, p_s[rhs])
        orhs = self.obj[N - 1]           # block 0: the objective row's RHS (xown)
        for q in range(npiv):
            # ---- ratio phase q: entering column, my rows' candidates ----
            if q == 0:
                c, zc, pc = c0, (self.obj[c0] if c0 >= 0 else 0.0), []
            else:
                tag = _tag(W, q - 1, ENTER)
                recs = _wait_all(lambda x: dev.enter[rank].get(x, (None,)), range(B),
                                 lambda v: v[0] == tag,
                                 f"rank {rank} block {b}: entering records of slot {q - 1}")
                win = _argmin([r[1] for r in recs])
                c, zc, pc = (win[2], win[3], win[4]) if win else (-1, 0.0, [])
            if c < 0:
                with lock:
                    sh["status"] = 0
                break
            key = None
            for i in rows:
                ig = self.row0 + i
                v = self.A[i, c]
                for s, (rs, cs, _) in enumerate(slots):
                    v = apply_sel(v, ig == rs, c == cs, fh[i][s], pc[s])
                if q > 0:
                    rs, cs, prhs = slots[-1]
                    bcur[i] = apply_sel(bcur[i], ig == rs, False, fh[i][-1], prhs)
                fh[i].append(v)
                if v > self.eps_piv:
                    ratio = bcur[i] / v
                    if not math.isnan(ratio):
                        t = int(bas[i]) if self.rule == "bland" else ig
                        k = (ratio, t, ig, list(fh[i]), bcur[i])
                        key = k if key is None or k[:2] < key[:2] else key
            self.delay("publish_ratio", rank, b, q)
            rec = (key, stop0)
            h = dev.half(it0, q)
            for d in range(nr):  # into EVERY rank's buffer (peer writes)
                dev.ratio[d][h][rank * B + b] = (_tag(W, q, RATIO), rec)
                self.delay("between_peer_writes", rank, b, q)
            with lock:
                for i in rows:
                    sh["f"].setdefault(q, {})[i] = fh[i][q]
            # ---- norm phase q: leaving row, p on my columns, entering key ----
            self.delay("poll_ratio", rank, b, q)
            tag = _tag(W, q, RATIO)
            recs = _wait_all(lambda x: dev.ratio[rank][h].get(x, (None,)), dev.slots,
                             lambda v: v[0] == tag,
                             f"rank {rank} block {b}: ratio records of slot {q}")
            if any(r[1][1] for r in recs):  # rank 0's stop request, seen by every rank here
                with lock:
                    sh["status"] = 1
                break
            cands = [(r[1][0], x) for x, r in enumerate(recs) if r[1][0] is not None]
            if not cands:
                with lock:
                    sh["status"] = 3
                break
            wk, wslot = min(cands, key=lambda t: t[0][:2])
            r, fr, rhs_r = wk[2], wk[3], wk[4]
            owner = wslot // B
            piv = fr[q]
            prhs = rhs_r / piv
            rl = r - dev.row0[owner]
            if dev.push and owner == rank:
                # owner-push: my stale row values into every peer's inbox (the
                # half of this pivot's parity), before my own slot work
                for d in range(nr):
                    if d != rank:
                        for j in cols:
                            dev.inbox[d][h][j] = (_tag(W, q, RATIO), self.A[rl, j])
                        self.delay("between_peer_writes", rank, b, q)
            self.delay("gather_row", rank, b, q, owner)
            if dev.push and owner != rank:
                tag_r = _tag(W, q, RATIO)
                box = dev.inbox[rank][h]
                got = _wait_all(lambda j: box.get(j, (None,)), cols, lambda v: v[0] == tag_r,
                                f"rank {rank} block {b}: pushed row of slot {q}")
                row = {j: v[1] for j, v in zip(cols, got)}
            else:
                src = dev.A[owner]  # the owner's stale rows (a peer pointer; my own rows)
                row = {j: src[rl, j] for j in cols}
            ekey = None
            for j in cols:
                v = row[j]
                for s, (rs, cs, _) in enumerate(slots):
                    v = apply_sel(v, r == rs, j == cs, fr[s], ph[j][s])
                p = v / piv
                ph[j].append(p)
                if j == c:
                    o[j] = 0.0
                elif p != 0.0:
                    o[j] = o[j] - zc * p
                if o[j] < -self.eps_opt:
                    ek = ((0.0 if self.rule == "bland" else o[j]), j, j, o[j], list(ph[j]))
                    ekey = ek if ekey is None or ek[:2] < ekey[:2] else ekey
            for i in rows:
                if self.row0 + i == r:
                    bas[i] = c
            if b == 0:
                orhs = apply_sel(orhs, False, False, zc, prhs)
            slots.append((r, c, prhs))
            dev.enter[rank][b] = (_tag(W, q, ENTER), ekey)
            with lock:
                sh["p"].setdefault(q, {}).update({j: ph[j][q] for j in cols})
                if b == 0:
                    sh["r"].append(r)
                    sh["c"].append(c)
                    sh["prhs"].append(prhs)
                    sh["made"] = q + 1
        # ---- window end: no rank may flush while a peer still gathers its rows ----
        # (owner-push: no peer reads my rows, so no barrier)
        if "no_done_barrier" not in dev.mutant and not dev.push:
            for d in range(nr):
                dev.done[d][rank * B + b] = _tag(W, 0, DONE)
            if b == 0:
                _wait_all(lambda x: dev.done[rank].get(x), range(nr * B),
                          lambda v: v == _tag(W, 0, DONE), f"rank {rank}: window-end barrier")
        with lock:
            for j in cols:
                obj_new[j] = o[j]
            if b == 0:
                obj_new[N - 1] = orhs

    # ---- the host loop (spx_solve): windows until a stop, reruns on ABORT ----
    def solve(self, max_iters):
        while self.status == 4 and self.it < max_iters:
            npiv = min(self.K, max_iters - self.it)
            if self.window(npiv) == "notres":
                self.reruns += 1
                self.epoch += 1  # the host's bump: the aborted window's words keep their verdict
        return self.status if self.status != 4 else 1
