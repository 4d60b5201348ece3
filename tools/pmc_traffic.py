"""Per-launch HBM traffic of the elimination kernel from two rocprofv3 --pmc
passes (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950).

Units/corrections per MI355X_MICROARCH.md §HBM: both counters are in KiB;
FETCH_SIZE reports half the bytes of a wide (16 B/lane) coalesced streaming
read on gfx950, so it is doubled; WRITE_SIZE is exact for 16-B stores.

usage: python tools/pmc_traffic.py FETCH_CSV WRITE_CSV KEY M_LOCAL TOUCHED_COLS OUT_JSON [K]
  K > 1: windowed mode, the kernel is flush_kernel (K pivots per launch)
"""
import csv
import json
import sys


def per_dispatch(path, counter, match="elim_kernel"):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if match in r["Kernel_Name"] and r["Counter_Name"] == counter]
    if not vals:
        raise SystemExit(f"no {counter} rows for {match} in {path}")
    return sum(vals) / len(vals), len(vals)


def main():
    fcsv, wcsv, key, m_local, cols, out = sys.argv[1:7]
    K = float(sys.argv[7]) if len(sys.argv) > 7 else 0.0
    m_local, cols = int(m_local), float(cols)
    match = "flush_" if K > 1 else "elim_kernel"  # flush_kernel or flush_lds_kernel
    f_kib, nf = per_dispatch(fcsv, "FETCH_SIZE", match)
    w_kib, nw = per_dispatch(wcsv, "WRITE_SIZE", match)
    fetch = 2.0 * f_kib * 1024.0
    write = w_kib * 1024.0
    if K > 1:
        alg = 16.0 * m_local * cols + 8.0 * K * (m_local + cols)
    else:
        alg = 16.0 * m_local * (cols - 1.0) + 8.0 * m_local
    try:
        data = json.load(open(out))
    except (OSError, ValueError):
        data = {}
    data[key] = {"kernel": match, "hbm_bytes_per_launch": fetch + write, "fetch_bytes": fetch,
                 "write_bytes": write, "alg_bytes_per_launch": alg,
                 "traffic_over_alg": (fetch + write) / alg, "dispatches": [nf, nw],
                 "raw_kib": {"FETCH_SIZE": f_kib, "WRITE_SIZE": w_kib},
                 "correction": "FETCH_SIZE x2 (gfx950 wide-read half count), KiB x1024"}
    json.dump(data, open(out, "w"), indent=1)
    print(json.dumps({key: data[key]}))


if __name__ == "__main__":
    main()
