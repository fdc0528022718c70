"""Per elimination level of the last factorization in a rocprofv3 kernel trace: fan-in / potrf / trsm
durations and grid sizes (workgroups), the gap to the next launch, and the time spent in levels whose
fan-in launch cannot fill the chip (< 256 workgroups) -- where the level-synchronous schedule is
latency-bound rather than MFMA-bound."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))


def wgs(r):
    g = int(r.get("Grid_Size", 0) or r.get("Grid_Size_X", 0) or 0)
    w = int(r.get("Workgroup_Size", 0) or r.get("Workgroup_Size_X", 0) or 1)
    return g // max(1, w)


def kname(r):
    n = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("viba::", "").split("<")[0]
    if n == "sntrsm_kernel":  # the two-column supernode schedule (VIBA_SUPERNODE=1)
        return "trsm_kernel"
    return "potrf_kernel" if n in ("potrf4_kernel", "potrf_trsm_kernel", "snpotrf_kernel", "snpotrf8_kernel",
                                   "snpotrf_trsm8_kernel") else n


ks = [(kname(r), int(r["Start_Timestamp"]), int(r["End_Timestamp"]), wgs(r)) for r in rows]
fam = ("fanin_kernel", "potrf_kernel", "trsm_kernel")
last_di = max(i for i, k in enumerate(ks) if k[0] == "diag_inverse_kernel")
first = last_di
while first > 0 and (ks[first - 1][0] in fam or ks[first - 1][0] == "copy_diag_kernel"):
    first -= 1
seg = ks[first:last_di + 1]
levels, cur = [], {}
for n, a, b, g in seg:
    if n == "fanin_kernel" and cur:
        levels.append(cur)
        cur = {}
    cur[n] = (a, b, g)
    if n == "diag_inverse_kernel":
        break
levels.append(cur)
t0 = seg[0][1]
small = [0.0, 0.0]
tot = {n: 0.0 for n in fam}
print(f"{'lvl':>4} {'start ms':>9} {'fanin us':>9} {'wg':>6} {'potrf us':>9} {'wg':>5} {'trsm us':>8} {'wg':>5} {'span us':>8}")
for i, L in enumerate(levels):
    a = min(v[0] for v in L.values())
    b = max(v[1] for v in L.values())
    d = {n: ((L[n][1] - L[n][0]) / 1e3 if n in L else 0.0) for n in fam}
    g = {n: (L[n][2] if n in L else 0) for n in fam}
    for n in fam:
        tot[n] += d[n]
    if g["fanin_kernel"] < 256:
        small[0] += (b - a) / 1e3
    else:
        small[1] += (b - a) / 1e3
    print(f"{i:4d} {(a - t0) / 1e6:9.3f} {d['fanin_kernel']:9.1f} {g['fanin_kernel']:6d} {d['potrf_kernel']:9.1f} "
          f"{g['potrf_kernel']:5d} {d['trsm_kernel']:8.1f} {g['trsm_kernel']:5d} {(b - a) / 1e3:8.1f}")
span = (seg[-1][2] - t0) / 1e3
print(f"factorization span {span / 1e3:.3f} ms; busy fan-in {tot['fanin_kernel'] / 1e3:.3f} potrf "
      f"{tot['potrf_kernel'] / 1e3:.3f} trsm {tot['trsm_kernel'] / 1e3:.3f} ms; levels with < 256 fan-in WGs "
      f"{small[0] / 1e3:.3f} ms, others {small[1] / 1e3:.3f} ms")
