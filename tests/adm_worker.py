"""Worker process for test_chain_admission_two_real_processes (GPU test
helper, not collected by pytest): one libspx process on GPU 0 beside another,
sharing the cross-process chain admission table (/dev/shm/spx_chain_<bus>).

usage: python tests/adm_worker.py ROLE SYNC_DIR BUDGET
  holder : enqueues a long Bland run (config-5 generator, 16 chain blocks)
           WITHOUT syncing, writes SYNC_DIR/holding, waits for SYNC_DIR/tried,
           then syncs and exits
  asker  : waits for SYNC_DIR/holding, solves 48 pivots (must be refused:
           the holder's 16 blocks + its 16 exceed BUDGET), writes
           SYNC_DIR/tried, waits for the holder to exit, solves again (must
           be admitted); prints one JSON line with both results' digests
"""
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "simplex-solver_amd"))

from simplex_amd import synth  # noqa: E402
from simplex_amd.engine import DeviceTableau  # noqa: E402


def wait_for(path, timeout=60.0):
    t0 = time.time()
    while not os.path.exists(path):
        if time.time() - t0 > timeout:
            raise SystemExit(f"timed out waiting for {path}")
        time.sleep(0.001)


def digest(e):
    return (hashlib.sha256(e.history().tobytes()).hexdigest(),
            hashlib.sha256(e.tableau().tobytes()).hexdigest())


def main():
    role, sync, budget = sys.argv[1], sys.argv[2], int(sys.argv[3])
    DeviceTableau.set_chain_budget(0, budget)
    T, basis = synth.full_tableau("degenerate", 2048, 2048, 5)  # N - 1 = 4096: 16 blocks
    with DeviceTableau(0) as e:
        e.set_window(24)
        e.load(T, basis)
        if role == "holder":
            e.run_pivots(24 * 400, rule="bland")  # ~100 ms of windows, no sync
            open(os.path.join(sync, "holding"), "w").close()
            wait_for(os.path.join(sync, "tried"))
            e.sync()
            print(json.dumps({"role": role, "stats": e.chain_stats()}))
            return
        wait_for(os.path.join(sync, "holding"))
        r1 = e.solve(rule="bland", max_iters=48)
        st1 = dict(e.chain_stats())
        d1 = digest(e)
        open(os.path.join(sync, "tried"), "w").close()
        wait_for(os.path.join(sync, "holder_done"))
        e.load(T, basis)
        r2 = e.solve(rule="bland", max_iters=48)
        st2 = dict(e.chain_stats())
        d2 = digest(e)
        print(json.dumps({"role": role, "iters": [r1.iters, r2.iters], "stats": [st1, st2],
                          "digests": [d1, d2]}))


if __name__ == "__main__":
    main()
