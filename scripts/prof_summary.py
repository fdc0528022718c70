"""Print the top kernels of a rocprofv3 --stats csv directory (default gpurun_out/prof_C)."""
import csv
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof_C"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 16
rows = list(csv.DictReader(open(f"{d}/run_kernel_stats.csv")))
for r in rows[:n]:
    print(f"{r['Name'][:58]:58s} calls {r['Calls']:>6s} avg {float(r['AverageNs'])/1e3:9.1f}us "
          f"tot {float(r['TotalDurationNs'])/1e6:8.2f}ms {r['Percentage'][:5]}%")
