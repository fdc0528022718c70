"""Factorization phase of the last LM iteration in a rocprofv3 kernel trace: per-kernel busy time,
the union of busy intervals (what the phase costs) and the idle gaps."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ks = [(r["Kernel_Name"].split("(")[0].replace("viba::", ""), int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
fam = ("fanin_kernel", "potrf_kernel", "trsm_kernel")
last_di = max(i for i, k in enumerate(ks) if k[0] == "diag_inverse_kernel")
first = last_di
while first > 0 and ks[first - 1][0] in fam:
    first -= 1
seg = ks[first:last_di]
t0, t1 = seg[0][1], max(k[2] for k in seg)
busy = {}
for n, a, b in seg:
    busy[n] = busy.get(n, 0) + (b - a)
iv = sorted((a, b) for _, a, b in seg)
union, cur_a, cur_b = 0, iv[0][0], iv[0][1]
for a, b in iv[1:]:
    if a > cur_b:
        union += cur_b - cur_a
        cur_a, cur_b = a, b
    else:
        cur_b = max(cur_b, b)
union += cur_b - cur_a
print(f"factor span {(t1 - t0) / 1e6:.2f} ms, union busy {union / 1e6:.2f} ms, launches {len(seg)}")
for n, v in busy.items():
    print(f"  {n:14s} busy {v / 1e6:.2f} ms")
