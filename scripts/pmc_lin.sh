#!/bin/bash
# PMC passes (one counter set per run) over the linearization kernels alone (scripts/kernel_probe.py),
# kernel-trace stats in a run of their own; summaries under gpurun_out/<tag>/
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-pmc_lin}
KS=${2:-10,12,13,14,15}
export TMPDIR=/tmp
mkdir -p $R/gpurun_out/$TAG
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$TAG/trace -o run -- python3 $R/scripts/kernel_probe.py C 3 fp64 $KS > $R/gpurun_out/$TAG/probe.json || exit $?
i=0
# PMC_SETS="set1;set2;..." replaces the default counter sets (each within one pass's block limits)
if [ -n "$PMC_SETS" ]; then IFS=';' read -ra SETS <<< "$PMC_SETS"; else
SETS=("SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY"
      "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS TCC_HIT_sum TCC_MISS_sum"
      "FETCH_SIZE" "WRITE_SIZE"); fi
for set in "${SETS[@]}"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $set --output-format csv -d $R/gpurun_out/$TAG/p$i -o run -- python3 $R/scripts/kernel_probe.py C 3 fp64 $KS > /dev/null || exit $?
done
cd $R && python3 - $TAG $i <<'PY'
import csv, glob, sys, collections
tag, n = sys.argv[1], int(sys.argv[2])
acc = collections.defaultdict(lambda: [0.0, 0])
for i in range(1, n + 1):
    for f in glob.glob(f"gpurun_out/{tag}/p{i}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = (r["Kernel_Name"].split("(")[0].replace("void ", "").replace("viba::", ""), r["Counter_Name"])
            acc[k][0] += float(r["Counter_Value"]); acc[k][1] += 1
with open(f"gpurun_out/{tag}/summary.txt", "w") as out:
    for (kn, cn), (v, c) in sorted(acc.items()):
        print(f"{kn[:40]:40s} {cn:22s} {v / c:.5g}", file=out)
PY
