"""Phase timing of one window's kernels (diagnostic; not part of the product).

Builds lib/libspx_probe.so with -DSPX_PHASE_TIMING (block 0 / thread 0 of every
window kernel stamps s_memrealtime, 100 MHz, at its phase boundaries), runs
windows on the config-3 tableau through it and prints, for the last window,
each kernel's phase times relative to the window start (us).

usage: python tools/probe_phases.py [--window 16] [--m 8192 --n 8192] [--build-only]
"""
import argparse
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "simplex-solver_amd")
LIB = os.path.join(PKG, "simplex_amd", "lib", "libspx_probe.so")


def build():
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
           "-shared", "-ffp-contract=off", "-mllvm", "-amdgpu-kernarg-preload-count=8",
           "-DSPX_PHASE_TIMING"] + (["-DSPX_PROBE_FINE"] if os.environ.get("SPX_PROBE_FINE") else []) + ["-o", LIB,
           os.path.join(PKG, "csrc", "spx_capi.hip"), "-lrccl"]
    subprocess.run(cmd, check=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--window", type=int, default=16)
    ap.add_argument("--m", type=int, default=8192)
    ap.add_argument("--n", type=int, default=8192)
    ap.add_argument("--build-only", action="store_true")
    ap.add_argument("--fmap", type=int, default=0)
    ap.add_argument("--chain", type=int, default=0, help="0 persistent chain, 1 lazy kernels")
    ap.add_argument("--fold", type=int, default=1, help="row_fix fold (spx_set_row_fix_fold)")
    a = ap.parse_args()
    if a.build_only or not os.path.exists(LIB):
        build()
        if a.build_only:
            return
    os.environ["SPX_LIB"] = LIB
    sys.path.insert(0, PKG)
    from simplex_amd import synth
    from simplex_amd.engine import DeviceTableau
    K = a.window
    Tf, obj, basis = synth.tableau_rows("dense", a.m, a.n, 20251205, order="F")
    e = DeviceTableau(0)
    e.set_window(K)
    e.set_chain(a.chain)
    e.set_row_fix_fold(bool(a.fold))
    e.load_rows(Tf, obj, basis, a.m, 0)
    e.set_elim_variant(0, 0, -1, flush_map=a.fmap & 3)
    del Tf
    e.run_pivots(4 * K)
    e.sync()
    # the last window's stamps stay in the buffer (one call: with the row_fix
    # fold, that window rewrites the previous window's leaving rows)
    e.run_pivots(3 * K)
    e.sync()
    lib = ctypes.CDLL(LIB)
    NB = 1024 + 2 * 8192
    buf = (ctypes.c_ulonglong * NB)()
    assert lib.spx_probe_read(buf, NB) == 0
    t = lambda slot, kind, ph: buf[((slot * 4 + kind) * 4 + ph) & 1023]
    t0 = t(0, 0, 0)
    us = lambda x: (x - t0) / 100.0
    if a.chain != 1 and t(K + 2, 0, 0):
        c0 = t(K + 2, 0, 0)
        fx = t(K + 2, 0, 1)
        print(f"chain entry -> slot 0: {(t0 - c0) / 100.0:6.2f} us (handshake passed at "
              f"{(t(K + 2, 0, 2) - c0) / 100.0:6.2f}" +
              (f", fold rows stored at {(fx - c0) / 100.0:6.2f}" if fx > c0 else "") + ")")
    names = ({0: "lazy_ratio", 1: "lazy_norm"} if a.chain == 1 else
             {0: "ratio ph.", 1: "norm ph."})
    print(f"window K={K}, m={a.m}, n={a.n}: us from lazy_ratio(0) entry (block 0, thread 0)")
    prev_end = None
    for q in range(K):
        for kind in (0, 1):
            ph = [us(t(q, kind, p)) for p in range(4)]
            gap = ph[0] - prev_end if prev_end is not None else 0.0
            print(f"q={q:2d} {names[kind]:10s} entry {ph[0]:8.2f} (+{gap:5.2f} after prev end)"
                  f"  phase1 +{ph[1]-ph[0]:5.2f}  phase2 +{ph[2]-ph[1]:5.2f}"
                  f"  end +{ph[3]-ph[2]:5.2f}  total {ph[3]-ph[0]:5.2f}")
            prev_end = ph[3]
            if a.chain != 1 and t(q, 2 + kind, 0) > t0:
                a0, a1 = us(t(q, 2 + kind, 0)), us(t(q, 2 + kind, 1))
                a2, a3 = us(t(q, 2 + kind, 2)), us(t(q, 2 + kind, 3))
                print(f"       fine: loads arrived +{a0 - ph[1]:5.2f}  slots applied "
                      f"+{a1 - a0:5.2f}  rest of phase2 +{ph[2] - a1:5.2f}  | end: argmin+lds "
                      f"+{a2 - ph[2]:5.2f}  barrier +{a3 - a2:5.2f}  publish +{ph[3] - a3:5.2f}")
                if t(q + 32, kind, 2) > t0:  # stamps inside the publish (SPX_PROBE_FINE)
                    p0, p1, p2 = (us(t(q + 32, kind, x)) for x in range(3))
                    print(f"       publish: key reduced +{p0 - a3:5.2f}  history read "
                          f"+{p1 - p0:5.2f}  stores issued +{p2 - p1:5.2f}  rest +{ph[3] - p2:5.2f}")
            if kind == 0 and os.environ.get("SPX_PROBE_FINE"):
                k0, k1 = us(t(q, 2, 0)), us(t(q, 2, 1))
                print(f"       fine: keys reduced +{k0 - ph[0]:5.2f}  wave_min +{k1 - k0:5.2f}")
    if a.chain != 1:
        nb = e.chain_blocks()
        cb = (ctypes.c_ulonglong * (32 * 8 * 256))()
        assert lib.spx_probe_read_chain(cb, 32 * 8 * 256) == 0
        ev = lambda q, k: [(cb[(q * 8 + k) * 256 + x] - t0) / 100.0 for x in range(nb)]
        import statistics as S
        print(f"per-block exchange timing ({nb} blocks), us: publish spread = last - first "
              "record stored; seen = poll done - last record stored (min / median / max)")
        for q in range(1, K - 1):
            for name, pub, see in (("ratio", 0, 1), ("enter", 2, 3)):
                P_, D_ = ev(q, pub), ev(q, see)
                last = max(P_)
                seen = [d - last for d in D_]
                print(f"  q={q:2d} {name}: publish spread {last - min(P_):5.2f} "
                      f"(block 0 at {P_[0] - min(P_):5.2f}, slowest block {P_.index(last):3d})  "
                      f"seen {min(seen):5.2f} / {S.median(seen):5.2f} / {max(seen):5.2f}")
    f0, f1 = us(t(K, 2, 0)), us(t(K, 2, 1))
    print(f"flush entry {f0:8.2f} (+{f0 - prev_end:5.2f})  block-0 duration {f1 - f0:7.2f}")
    rch, G = ctypes.c_int(), ctypes.c_int()
    lib.spx_probe_flush_grid.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int),
                                         ctypes.POINTER(ctypes.c_int)]
    lib.spx_probe_flush_grid(e._ctx, ctypes.byref(rch), ctypes.byref(G))
    nblk = min(rch.value * G.value, 8192)
    import numpy as np
    st = np.array([buf[1024 + 2 * b] for b in range(nblk)], dtype=np.float64)
    en = np.array([buf[1024 + 2 * b + 1] for b in range(nblk)], dtype=np.float64)
    st, en = (st - t0) / 100.0 - f0, (en - t0) / 100.0 - f0
    dur = en - st
    print(f"flush grid {rch.value} row chunks x {G.value} groups = {nblk} blocks")
    q = lambda a: " ".join(f"{x:7.1f}" for x in np.percentile(a, [0, 10, 50, 90, 100]))
    print(f"  block start  pct 0/10/50/90/100: {q(st)}")
    print(f"  block end    pct 0/10/50/90/100: {q(en)}")
    print(f"  block dur    pct 0/10/50/90/100: {q(dur)}")
    g = np.arange(nblk) // rch.value
    gd = np.array([dur[g == k].mean() for k in range(G.value)])
    print(f"  per-group mean dur min/median/max: {gd.min():.1f} {np.median(gd):.1f} {gd.max():.1f}")
    ch = np.arange(nblk) % rch.value
    cd = np.array([dur[ch == k].mean() for k in range(rch.value)])
    print("  per-chunk mean dur:", " ".join(f"{x:.0f}" for x in cd))
    xcd = np.arange(nblk) % 8
    print("  per-XCD mean dur:", " ".join(f"{dur[xcd == k].mean():.0f}" for k in range(8)))
    # row_fix (block 0 stamps, every block's entry / exit) after the flush's last block
    r0 = us(t(K + 1, 0, 0))
    if r0 > 0:
        fl_end = en.max() + f0
        rb = [(buf[1024 + 2 * (4096 + b)], buf[1024 + 2 * (4096 + b) + 1]) for b in range(4096)]
        rb = np.array([(us(a_), us(b_)) for a_, b_ in rb if a_ > t0])
        print(f"row_fix: entry {r0 - fl_end:+6.2f} us after the flush's last block; block 0: "
              f"round 1 +{us(t(K + 1, 0, 1)) - r0:5.2f}  round 2 +{us(t(K + 1, 0, 2)) - us(t(K + 1, 0, 1)):5.2f}"
              f"  lastL+barrier +{us(t(K + 1, 1, 2)) - us(t(K + 1, 0, 2)):5.2f}"
              f"  chains +{us(t(K + 1, 1, 1)) - us(t(K + 1, 1, 2)):5.2f}"
              f"  store issue +{us(t(K + 1, 0, 3)) - us(t(K + 1, 1, 1)):5.2f}"
              f"  stores drained +{us(t(K + 1, 1, 0)) - us(t(K + 1, 0, 3)):5.2f}")
        if len(rb):
            print(f"  {len(rb)} blocks: entry pct 0/50/100 {q(rb[:, 0] - r0)}  exit pct {q(rb[:, 1] - r0)}")
    if hasattr(lib, "spx_probe_read_wave"):
        wb = (ctypes.c_ulonglong * (2 * 4 * 8192))()
        assert lib.spx_probe_read_wave(wb, 2 * 4 * 8192) == 0
        raw = np.frombuffer(wb, dtype=np.uint64).reshape(8192, 4, 2)[:nblk]
        wend = (raw[:, :, 0].astype(np.float64) - t0) / 100.0 - f0  # us from flush entry
        info = raw[:, :, 1]
        live = raw[:, :, 0] > 0
        hw = (info & np.uint64(0xffffffff)).astype(np.int64)
        xc = ((info >> np.uint64(32)) & np.uint64(0xff)).astype(np.int64)
        cols = (info >> np.uint64(40)).astype(np.int64)
        cu = (xc << 16) | ((hw >> 8) & 0xff)  # XCC, SE/SH/CU bits of HW_ID
        wdur = wend - st[:, None]
        print(f"  waves: {live.sum()} live; end pct 0/10/50/90/100: {q(wend[live])}")
        print("  per-wave-index mean end:", " ".join(f"{wend[:, w][live[:, w]].mean():.1f}"
                                                     for w in range(4)))
        ucu = np.unique(cu[live])
        cu_end = np.array([wend[live & (cu == c)].max() for c in ucu])
        cu_nb = np.array([len(np.unique(np.nonzero(live & (cu == c))[0])) for c in ucu])
        print(f"  CUs {len(ucu)}; blocks per CU {np.bincount(cu_nb)}; per-CU last wave end "
              f"pct 0/10/50/90/100: {q(cu_end)}")
        us_per_col = wdur[live] / np.maximum(cols[live], 1)
        print(f"  us per column per wave pct 0/10/50/90/100: {q(us_per_col)}")
        gmean = np.array([wdur[(g == k)[:, None] & live].mean() for k in range(G.value)])
        order = np.argsort(gmean)
        print("  fastest groups:", " ".join(f"{k}:{gmean[k]:.0f}" for k in order[:8]))
        print("  slowest groups:", " ".join(f"{k}:{gmean[k]:.0f}" for k in order[-8:]))
        out = os.environ.get("PROBE_NPZ")
        if out:
            np.savez(out, st=st, en=en, wend=wend, hw=hw, xc=xc, cols=cols, live=live,
                     rch=rch.value, G=G.value)
    e.close()


if __name__ == "__main__":
    main()
