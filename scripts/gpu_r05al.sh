#!/bin/bash
# SQ counters of the fan-in: target pairs (fanin_kernel2) against single targets (fanin_kernel); and the
# target-pair parity test
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=r05al
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_supernode_gpu.py -k target_pairs > gpurun_out/pytest_${T}.log 2>&1 || { tail -30 gpurun_out/pytest_${T}.log; exit 1; }
tail -1 gpurun_out/pytest_${T}.log
C="SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_VALU_MFMA_BUSY_CYCLES,SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE,SQ_WAIT_INST_LDS"
cd /tmp
for P in 1 0; do
  (VIBA_FAN_PAIRS=$P timeout -s KILL 240 rocprofv3 --pmc $C --kernel-include-regex "fanin_kernel" --output-format csv -d $R/gpurun_out/sq_${T}_p$P -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-banded-count --profile-steps 1 > /dev/null 2> $R/gpurun_out/sq_${T}_p$P.log) || { tail -5 $R/gpurun_out/sq_${T}_p$P.log; exit 1; }
done
cd $R
python - <<'PY'
import csv, glob, collections
for P in (1, 0):
    f = glob.glob(f"gpurun_out/sq_r05al_p{P}/**/*counter_collection.csv", recursive=True)[0]
    tot = collections.defaultdict(float); n = collections.Counter()
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0]
        tot[(k, r["Counter_Name"])] += float(r["Counter_Value"]); n[(k, r["Counter_Name"])] += 1
    for k in sorted({a for a, _ in tot}):
        d = {c: tot[(kk, c)] for kk, c in tot if kk == k}
        w = d.get("SQ_WAVE_CYCLES", 1)
        print(P, k, {c: round(v / w, 3) for c, v in d.items() if c != "SQ_WAVE_CYCLES"}, "wave_cycles", w)
PY
