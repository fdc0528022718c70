"""Per kernel of a rocprofv3 --kernel-trace csv: dispatches, average duration, and busy time -- the union of
the dispatches' [start, end] intervals, which is what bench.py's roofline divides by when launches of one
kernel overlap (the factorization's streams).  Usage:

    python scripts/busy_union.py gpurun_out/prof_X/run_kernel_trace.csv [name-substring ...]
"""
import csv
import json
import sys


def busy(intervals):
    total, end = 0, None
    for a, b in sorted(intervals):
        if end is None or a > end:
            total += b - a
            end = b
        elif b > end:
            total += b - end
            end = b
    return total


def main():
    path = sys.argv[1]
    want = sys.argv[2:] or ["fanin_kernel"]
    rows = list(csv.DictReader(open(path)))
    out = {}
    for w in want:
        iv = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows if w in r["Kernel_Name"]]
        if not iv:
            continue
        n = len(iv)
        out[w] = {"dispatches": n, "avg_us": sum(b - a for a, b in iv) / n / 1e3,
                  "busy_us_per_dispatch": busy(iv) / n / 1e3, "busy_ms_total": busy(iv) / 1e6}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
