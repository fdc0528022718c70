"""Print one LM iteration's kernel timeline from a rocprofv3 kernel trace (the last full iteration)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
seq = [(r["Kernel_Name"].split("(")[0].replace("viba::", "").replace("void ", ""),
        (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3, int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
       for r in rows]
idx = [i for i, s in enumerate(seq) if s[0] == "boxplus_reduced_kernel"]
a, b = idx[-2], idx[-1]
out = []
for n, dur, t, e in seq[a + 1:b + 1]:
    if out and out[-1][0] == n:
        out[-1][1] += dur; out[-1][2] += 1; out[-1][4] = e
    else:
        out.append([n, dur, 1, t, e])
t0 = out[0][3]
fan = [0.0, 0]
for n, dur, c, t, e in out:
    if n.split("<")[0] in ("fanin_kernel", "potrf_kernel", "trsm_kernel", "potrf4_kernel", "potrf_trsm_kernel"):
        fan[0] += dur; fan[1] += c
        continue
    print(f"{(t - t0) / 1e6:8.2f}ms {n:32s} x{c:4d} busy {dur / 1e3:7.3f} ms span {(e - t) / 1e6:7.3f}")
print(f"factor kernels busy {fan[0] / 1e3:.3f} ms over {fan[1]} launches; iteration span {(out[-1][4] - t0) / 1e6:.2f} ms")
