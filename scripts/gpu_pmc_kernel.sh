#!/bin/bash
# PMC passes (one counter group per pass) over the kernels matching $1; per-kernel averages printed
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp VIBA_NO_GRAPHS=1
R=$GRAFT_REPO_ROOT
RE=$1
shift
cd /tmp
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -k 10 400 rocprofv3 --pmc $grp --kernel-include-regex "$RE" --output-format csv -d $R/gpurun_out/pmck_$i -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline > /dev/null 2> $R/gpurun_out/pmck_$i.log || exit $?
done
cd $R && python3 - "$i" <<'PY'
import csv, glob, sys, collections
n = int(sys.argv[1])
for i in range(1, n + 1):
    for f in glob.glob(f"gpurun_out/pmck_{i}/**/*counter_collection.csv", recursive=True):
        acc = collections.defaultdict(lambda: [0.0, 0])
        for r in csv.DictReader(open(f)):
            k = (r["Kernel_Name"].split("(")[0], r["Counter_Name"])
            acc[k][0] += float(r["Counter_Value"]); acc[k][1] += 1
        for (kn, cn), (v, c) in sorted(acc.items()):
            print(f"{kn[:40]:40s} {cn:28s} avg/dispatch-row {v / c:.4g}  rows {c}")
PY
