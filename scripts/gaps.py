"""Device idle inside the timed iterations of a rocprofv3 kernel trace: the union of kernel intervals
between two LM iteration boundaries (boxplus_reduced_kernel launches), its idle gaps, and the largest
gaps with the kernels either side.

    python scripts/gaps.py gpurun_out/<dir>/run_kernel_trace.csv [iterations=3] [top=12]
"""
import csv
import sys


def main():
    path = sys.argv[1]
    n_it = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 12
    rows = list(csv.DictReader(open(path)))
    ev = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                  r["Kernel_Name"].split("(")[0].replace("viba::", "").replace("void ", "")) for r in rows))
    marks = [i for i, e in enumerate(ev) if e[2] == "boxplus_reduced_kernel"]
    if len(marks) < n_it + 1:
        sys.exit(f"only {len(marks)} iteration boundaries in the trace")
    a, b = marks[-n_it - 1], marks[-1]
    seg = ev[a:b]
    busy, gaps, cur_end, prev_name = 0, [], seg[0][0], seg[0][2]
    for s, e, name in seg:
        if s > cur_end:
            gaps.append((s - cur_end, prev_name, name, cur_end))
        if e > cur_end:
            busy += e - max(s, cur_end)
            cur_end, prev_name = e, name
    span = cur_end - seg[0][0]
    idle = sum(g[0] for g in gaps)
    print(f"{n_it} iterations: span {span / 1e6:.3f} ms ({span / 1e6 / n_it:.3f} per iteration), busy {busy / 1e6:.3f} ms, "
          f"idle {idle / 1e6:.3f} ms ({idle / 1e6 / n_it:.3f} per iteration) in {len(gaps)} gaps")
    for g, p, n, t in sorted(gaps, reverse=True)[:top]:
        print(f"  {g / 1e3:8.1f} us at {(t - seg[0][0]) / 1e6:8.3f} ms: after {p:34s} before {n}")


if __name__ == "__main__":
    main()
