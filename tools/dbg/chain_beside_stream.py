"""Diagnostic: the persistent chain's per-pivot time alone and beside an HBM
read-modify-write stream running on a CU-masked stream (tools/dbg/
stream_beside.hip), at config 3.  Answers whether overlapping a window's
chain with the previous window's flush could pay."""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "simplex-solver_amd"))
from simplex_amd import synth  # noqa: E402
from simplex_amd.engine import DeviceTableau  # noqa: E402

sb = ctypes.CDLL(os.path.join(ROOT, "tools", "dbg", "libstream_beside.so"))
sb.sb_init.argtypes = [ctypes.c_int, ctypes.c_int64]
sb.sb_time.restype = ctypes.c_double
K = int(os.environ.get("CB_WINDOW", "16"))
m = n = 8192
Tf, obj, basis = synth.tableau_rows("dense", m, n, 20251205, order="F")
e = DeviceTableau(0)
e.set_window(K)
e.load_rows(Tf, obj, basis, m, 0)
del Tf
e.run_pivots(4 * K)
e.sync()


def chain_us(windows=8):
    e.set_chain_timing(True)
    e.run_pivots(windows * K)
    e.sync()
    ms, cnt = e.chain_timing(reset=True)
    e.set_chain_timing(False)
    return 1e3 * ms / (cnt * K)


for every in (int(x) for x in os.environ.get("CB_EVERY", "4,2").split(",")):
    on = sb.sb_init(every, 1 << 30)
    alone_ms = sb.sb_time(20) / 20
    base = chain_us()
    sb.sb_run(4000)  # ~0.5 s of stream, longer than the chain windows below
    time.sleep(0.002)
    beside = chain_us()
    busy = sb.sb_query() == 0
    sb.sb_sync()
    print(json.dumps({"window": K, "stream_cus": on, "stream_pass_ms_alone": alone_ms,
                      "stream_TBps_alone": 2 * (1 << 30) / (alone_ms * 1e-3) / 1e12,
                      "chain_us_per_pivot_alone": base, "chain_us_per_pivot_beside": beside,
                      "stream_still_running": busy}), flush=True)
e.close()
