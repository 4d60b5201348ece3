"""Gaps between the launches of a window in a rocprofv3 kernel trace
(--kernel-trace CSV): chain -> flush -> row_fix -> next window's chain, the
medians over the trace's steady windows (kernel names by substring).

  python tools/trace_gaps.py gpurun_out/trace/prof/<host>/<pid>/bench_kernel_trace.csv
"""
import csv
import statistics
import sys


def main(path):
    rows = list(csv.DictReader(open(path)))
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
                 for r in rows if r.get("Kind", "KERNEL_DISPATCH") == "KERNEL_DISPATCH"))
    kind = lambda n: ("chain" if "chain_kernel" in n else "flush" if "flush_lds" in n
                      else "row_fix" if "row_fix" in n else None)
    seq = [(s, e, kind(n)) for s, e, n in ks if kind(n)]
    gaps = {}
    durs = {}
    for (s0, e0, k0), (s1, e1, k1) in zip(seq, seq[1:]):
        gaps.setdefault(f"{k0} -> {k1}", []).append((s1 - e0) / 1e3)
    for s, e, k in seq:
        durs.setdefault(k, []).append((e - s) / 1e3)
    out = {"kernels": {k: {"n": len(v), "median_us": round(statistics.median(v), 2)}
                       for k, v in durs.items()},
           "gaps_us": {k: {"n": len(v), "median": round(statistics.median(v), 2),
                           "p10": round(sorted(v)[len(v) // 10], 2),
                           "p90": round(sorted(v)[9 * len(v) // 10], 2)}
                       for k, v in gaps.items() if len(v) >= 5}}
    import json
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
