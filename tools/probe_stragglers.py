"""Which chain blocks publish last, and why (diagnostic; not part of the product).

VERDICT r4 "do this" 2(a): the slowest of the chain's B blocks publishes its
record ~0.7 us after the first, and every block waits for it.
This tool runs many windows of the config-3 chain through the probe build
(-DSPX_PHASE_TIMING: every block's thread 0 stamps s_memrealtime at 8 points
of each phase, spx_chain.hpp SPX_PROBE_CHAIN*) and asks whether the straggler
is systematic -- the same blocks every time, the RHS-owning last block, blocks
holding slack (basic) columns, blocks on one XCD -- and which part of its phase
made it late:

  start   the block saw the previous exchange's winner late (poll done)
  gather  its dependent loads (stale tableau value + the winner's history)
  slots   applying the window's pending slots
  rest    argmin, LDS hand-off, barrier, block key and the record stores

Per (window, slot, phase) the lateness of block b is its record-store time
minus the median block's; the components are split the same way.  Output: a
text report (stdout) and, with --npz, the raw stamps.

usage: python tools/probe_stragglers.py [--windows 40] [--window 24] [--npz out.npz]
"""
import argparse
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "simplex-solver_amd")
LIB = os.path.join(PKG, "simplex_amd", "lib", "libspx_probe.so")
EV = 8  # spx_chain.hpp PROBE_CHAIN_EV


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--window", type=int, default=24)
    ap.add_argument("--windows", type=int, default=40)
    ap.add_argument("--warm", type=int, default=4)
    ap.add_argument("--m", type=int, default=8192)
    ap.add_argument("--n", type=int, default=8192)
    ap.add_argument("--npz", default="")
    a = ap.parse_args()
    if not os.path.exists(LIB):
        raise SystemExit(f"{LIB} missing: python tools/probe_phases.py --build-only")
    os.environ["SPX_LIB"] = LIB
    sys.path.insert(0, PKG)
    from simplex_amd import synth
    from simplex_amd.engine import DeviceTableau
    K = a.window
    Tf, obj, basis = synth.tableau_rows("dense", a.m, a.n, 20251205, order="F")
    e = DeviceTableau(0)
    e.set_window(K)
    e.load_rows(Tf, obj, basis, a.m, 0)
    del Tf
    lib = ctypes.CDLL(LIB)
    e.run_pivots(a.warm * K)
    e.sync()
    B = e.chain_blocks()
    NB = 32 * EV * 256
    stamps = np.zeros((a.windows, K, EV, B), dtype=np.float64)
    hw = (ctypes.c_ulonglong * 256)()
    for w in range(a.windows):
        e.run_pivots(K)
        e.sync()
        buf = (ctypes.c_ulonglong * NB)()
        assert lib.spx_probe_read_chain(buf, NB) == 0
        raw = np.frombuffer(buf, dtype=np.uint64).reshape(32, EV, 256)[:K, :, :B]
        stamps[w] = raw.astype(np.float64) / 100.0  # us
        if w == 0:
            assert lib.spx_probe_read_chain_hw(hw, 256) == 0
    hist = e.history()
    N = a.n + a.m + 1
    cpb = (N - 1 + B - 1) // B
    rpb = (a.m + B - 1) // B
    e.close()
    hwv = np.frombuffer(hw, dtype=np.uint64)[:B]
    xcc = ((hwv >> np.uint64(32)) & np.uint64(0xf)).astype(int)
    cu = ((hwv >> np.uint64(8)) & np.uint64(0xff)).astype(int)  # SE / SH / CU bits of HW_ID
    print(f"config {a.m}x{a.n}, K={K}, {a.windows} windows, {B} blocks "
          f"({cpb} columns, {rpb} rows each)")
    print("block -> XCC:", " ".join(str(x) for x in xcc))
    it0 = len(hist) - a.windows * K
    rows = hist[it0:, 0].reshape(a.windows, K)
    cols = hist[it0:, 1].reshape(a.windows, K)

    # phases: (name, start event (slot offset), loads, slots, record)
    comps = {}
    for name in ("ratio", "norm"):
        S, L, SL, R = [], [], [], []
        for q in range(1, K - 1):
            if name == "ratio":
                s, ld, sl, rc = stamps[:, q - 1, 3], stamps[:, q, 4], stamps[:, q, 6], stamps[:, q, 0]
            else:
                s, ld, sl, rc = stamps[:, q, 1], stamps[:, q, 5], stamps[:, q, 7], stamps[:, q, 2]
            S.append(s), L.append(ld), SL.append(sl), R.append(rc)
        S, L, SL, R = (np.stack(x, 1) for x in (S, L, SL, R))  # [window, q, block]
        comps[name] = (S, L, SL, R)

    def med(x):
        return np.median(x, axis=-1, keepdims=True)

    for name, (S, L, SL, R) in comps.items():
        late = R - med(R)
        parts = {"start": S - med(S),
                 "gather": (L - S) - med(L - S),
                 "slots": (SL - L) - med(SL - L),
                 "rest": (R - SL) - med(R - SL)}
        spread = (R.max(-1) - R.min(-1))
        p50 = (R.max(-1) - np.median(R, -1))
        print(f"\n== {name} phase (slots 1..{K - 2}, {R.shape[0] * R.shape[1]} exchanges) ==")
        print(f"record spread last-first: mean {spread.mean():.2f} us, last-median "
              f"{p50.mean():.2f} us; phase (median block) start->record {np.median(R - S):.2f} us: "
              f"gather {np.median(L - S):.2f}, slots {np.median(SL - L):.2f}, "
              f"rest {np.median(R - SL):.2f}")
        last = R.argmax(-1)
        cnt = np.bincount(last.ravel(), minlength=B)
        order = np.argsort(-cnt)
        n_ex = last.size
        print(f"last publisher: uniform would be {100.0 / B:.1f}% each; top blocks:",
              " ".join(f"b{b}:{100.0 * cnt[b] / n_ex:.0f}%(x{xcc[b]})" for b in order[:8]))
        # what made the last publisher late (its components vs the median block)
        w_i, q_i = np.meshgrid(np.arange(R.shape[0]), np.arange(R.shape[1]), indexing="ij")
        lp = {k: v[w_i, q_i, last] for k, v in parts.items()}
        print("the last publisher's lateness (mean us vs the median block): total "
              f"{late[w_i, q_i, last].mean():.2f} = " +
              " + ".join(f"{k} {v.mean():.2f}" for k, v in lp.items()))
        dom = np.argmax(np.stack([lp[k] for k in parts], 0), 0)
        print("dominant component of the last publisher's lateness:",
              " ".join(f"{k} {100.0 * np.mean(dom == x):.0f}%" for x, k in enumerate(parts)))
        # systematic? per-block mean lateness and its spread over blocks
        pb = late.mean((0, 1))
        print(f"per-block mean lateness: min {pb.min():.2f} median {np.median(pb):.2f} "
              f"max {pb.max():.2f} us (b{pb.argmax()}); stdev over exchanges "
              f"{late.std():.2f}, over block means {pb.std():.2f}")
        for k, v in parts.items():
            m_ = v.mean((0, 1))
            print(f"  {k:6s} per-block mean: min {m_.min():+.2f} max {m_.max():+.2f} "
                  f"(b{m_.argmax()}), by XCC: " +
                  " ".join(f"{x}:{m_[xcc == x].mean():+.2f}" for x in sorted(set(xcc))))
        print("  lateness by XCC:", " ".join(f"{x}:{pb[xcc == x].mean():+.2f}"
                                             for x in sorted(set(xcc))))
        half = B // 2
        print(f"  lateness blocks 0..{half - 1} (structural columns) {pb[:half].mean():+.2f}, "
              f"{half}..{B - 1} (slack columns) {pb[half:].mean():+.2f}, last block "
              f"{pb[-1]:+.2f}")
        # the block owning the leaving row (ratio) / the entering column (norm)
        if name == "ratio":
            own = np.stack([rows[:, q] // rpb for q in range(1, K - 1)], 1)
        else:
            own = np.stack([cols[:, q + 1] // cpb for q in range(1, K - 1)], 1)
        ol = late[w_i, q_i, np.clip(own, 0, B - 1)]
        print(f"  the block owning the {'leaving row' if name == 'ratio' else 'next entering column'}"
              f": lateness {ol.mean():+.2f} us, last {100.0 * np.mean(own == last):.0f}% of the time")
        # seen: next phase's start minus this phase's last record
    S_n = comps["norm"][0]
    R_r = comps["ratio"][3]
    seen_r = S_n - R_r.max(-1, keepdims=True)
    S_r = comps["ratio"][0][:, 1:]
    R_n = comps["norm"][3][:, :-1]
    seen_n = S_r - R_n.max(-1, keepdims=True)
    print(f"\nseen (poll done - last record): ratio min/median/max "
          f"{seen_r.min():.2f}/{np.median(seen_r):.2f}/{seen_r.max():.2f}, "
          f"enter {seen_n.min():.2f}/{np.median(seen_n):.2f}/{seen_n.max():.2f} us")
    print("seen by XCC (median):", " ".join(
        f"{x}:{np.median(seen_r[..., xcc == x]):.2f}/{np.median(seen_n[..., xcc == x]):.2f}"
        for x in sorted(set(xcc))))
    if a.npz:
        np.savez(a.npz, stamps=stamps, xcc=xcc, cu=cu, hist=hist[it0:], B=B, cpb=cpb, rpb=rpb)


if __name__ == "__main__":
    main()
