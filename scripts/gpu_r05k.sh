#!/bin/bash
# supernode stream groups: group balance, parity, bench A/B (1 stream / 4 eager / 4 graph)
set -o pipefail
mkdir -p gpurun_out
T=r05k
VIBA_SCHUR_STATS=0 timeout -k 10 300 python scripts/symbolic_stats.py C > gpurun_out/sym_$T.log 2>&1 || { tail -5 gpurun_out/sym_$T.log; exit 1; }
grep "stream group" gpurun_out/sym_$T.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_supernode_gpu.py tests/test_parity_gpu.py > gpurun_out/pytest_$T.log 2>&1 || { tail -30 gpurun_out/pytest_$T.log; exit 1; }
tail -2 gpurun_out/pytest_$T.log
for cfg in "VIBA_SN_STREAMS=1" "VIBA_SN_STREAMS=4" "VIBA_SN_STREAMS=4 VIBA_SN_GRAPH=1" "VIBA_SN_STREAMS=2" "VIBA_SN_STREAMS=1"; do
  n=$(echo $cfg | tr ' =' '__')
  env $cfg timeout -k 10 300 python bench.py --no-cpu-baseline --no-banded-count --profile-family -1 > gpurun_out/bench_${T}_$n.json 2> gpurun_out/bench_${T}_$n.log || { tail -20 gpurun_out/bench_${T}_$n.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/bench_${T}_$n.json').read().strip().splitlines()[-1]); print('$cfg', round(d['value'],2), d['phases_ms'])"
done
