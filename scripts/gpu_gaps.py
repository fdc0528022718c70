"""Idle intervals of the GPU in a rocprofv3 kernel trace: the union of every kernel's [start, end) over all
queues, per LM iteration of the timed region (iterations cut at the schur_run4 launches), and the
largest gaps with the kernels on either side.  Usage: python scripts/gpu_gaps.py run_kernel_trace.csv"""
import csv
import sys
from collections import Counter


def main(path, top=25):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0]))
    rows.sort()
    cuts = [s for s, e, n in rows if "schur_run4" in n]
    if len(cuts) < 3:
        print("fewer than 3 iterations in the trace")
        return
    # steady-state iterations: between consecutive schur launches, skipping the first
    tot_busy = tot_span = 0
    gaps = Counter()
    big = []
    for a, b in zip(cuts[1:-1], cuts[2:]):
        ev = [(s, e, n) for s, e, n in rows if a <= s < b]
        busy = 0
        cur_s, cur_e, cur_n = ev[0]
        for s, e, n in ev[1:]:
            if s > cur_e:
                busy += cur_e - cur_s
                g = s - cur_e
                key = f"{cur_n} -> {n}"
                gaps[key] += g
                big.append((g, key))
                cur_s, cur_e, cur_n = s, e, n
            elif e > cur_e:
                cur_e, cur_n = e, n
        busy += cur_e - cur_s
        tot_busy += busy
        tot_span += b - a
    nit = len(cuts) - 2
    print(f"{nit} iterations: span {tot_span / nit / 1e6:.3f} ms, GPU busy {tot_busy / nit / 1e6:.3f} ms, "
          f"idle {(tot_span - tot_busy) / nit / 1e6:.3f} ms per iteration")
    print("idle per iteration by transition (us):")
    for k, v in gaps.most_common(top):
        print(f"  {v / nit / 1e3:8.1f}  {k}")


if __name__ == "__main__":
    main(sys.argv[1])
