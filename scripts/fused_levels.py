"""Per-level durations of factor_level_kernel in the last factorization of a rocprofv3 kernel trace,
beside the 3-launch level spans of an older trace's level_profile output (optional second argument)."""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
ks = [(r["Kernel_Name"].split("(")[0].replace("viba::", ""), int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
       int(r.get("Grid_Size", 0) or r.get("Grid_Size_X", 0)) // max(1, int(r.get("Workgroup_Size", 0) or r.get("Workgroup_Size_X", 1))))
      for r in rows]
last = max(i for i, k in enumerate(ks) if k[0] == "diag_inverse_kernel")
first = last
while first > 0 and ks[first - 1][0] == "factor_level_kernel":
    first -= 1
seg = ks[first:last]
old = {}
if len(sys.argv) > 2:
    for line in open(sys.argv[2]):
        f = line.split()
        if f and f[0].isdigit():
            old[int(f[0])] = float(f[-1])
tot = sum(b - a for _, a, b, _ in seg) / 1e3
span = (seg[-1][2] - seg[0][1]) / 1e3
print(f"levels {len(seg)}: busy {tot / 1e3:.3f} ms, span {span / 1e3:.3f} ms")
for i, (n, a, b, g) in enumerate(seg):
    gap = (seg[i + 1][1] - b) / 1e3 if i + 1 < len(seg) else 0.0
    print(f"{i:4d} {(b - a) / 1e3:9.1f} us  wg {g:6d}  gap {gap:6.1f}  old span {old.get(i, 0):8.1f}")
