"""Concurrency profile of the last factorization in a rocprofv3 kernel trace (the kernels between the last
Schur tile-product launch and the last diagonal-tile inverse): span, and the time during which each set
of kernel kinds was running -- e.g. how long only diagonal blocks / rows ran with no fan-in beside them.

    python scripts/factor_overlap.py gpurun_out/prof_X/run_kernel_trace.csv
"""
import collections
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    name = lambda r: r["Kernel_Name"].split("(")[0].replace("viba::", "")  # noqa: E731
    idx = [i for i, r in enumerate(rows) if "diag_inverse" in r["Kernel_Name"]]
    b = idx[-1]
    a = [i for i in range(b) if "schur_run4" in rows[i]["Kernel_Name"]][-1]
    fac = rows[a + 1:b + 1]
    t0 = int(fac[0]["Start_Timestamp"])
    ev = []
    for r in fac:
        ev.append((int(r["Start_Timestamp"]) - t0, 1, name(r)))
        ev.append((int(r["End_Timestamp"]) - t0, -1, name(r)))
    ev.sort()
    kinds, last, prof = collections.Counter(), 0, collections.Counter()
    for t, d, n in ev:
        prof[tuple(sorted(k for k, c in kinds.items() if c > 0))] += t - last
        last = t
        kinds[n] += d
    print(f"span {(int(fac[-1]['End_Timestamp']) - t0) / 1e6:.3f} ms, {len(fac)} launches on queues "
          f"{dict(collections.Counter(r['Queue_Id'] for r in fac))}")
    for k, v in sorted(prof.items(), key=lambda x: -x[1]):
        print(f"{v / 1e6:7.3f} ms  {' + '.join(k) if k else '(idle)'}")


if __name__ == "__main__":
    main()
