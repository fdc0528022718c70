#!/bin/bash
# staged observation-group kernel: parity, solo times (new / old), bench A/B
set -o pipefail
mkdir -p gpurun_out
T=r05j
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_parity_gpu.py tests/test_parity_configs.py > gpurun_out/pytest_$T.log 2>&1 || { tail -30 gpurun_out/pytest_$T.log; exit 1; }
tail -3 gpurun_out/pytest_$T.log
VIBA_SCHUR_STATS=1 timeout -k 10 300 python scripts/kernel_probe.py C 1 fp64 14 > /dev/null 2> gpurun_out/schurstats_$T.log || exit 1
grep "schur stats" gpurun_out/schurstats_$T.log
timeout -k 10 300 python scripts/kernel_probe.py C 5 fp64,mixed 12,13,14 > gpurun_out/probe_${T}_new.json 2> gpurun_out/probe_${T}_new.log || { tail -5 gpurun_out/probe_${T}_new.log; exit 1; }
cat gpurun_out/probe_${T}_new.json
VIBA_GROUPS_V=1 timeout -k 10 300 python scripts/kernel_probe.py C 5 fp64 13 > gpurun_out/probe_${T}_old.json 2> gpurun_out/probe_${T}_old.log || { tail -5 gpurun_out/probe_${T}_old.log; exit 1; }
cat gpurun_out/probe_${T}_old.json
for v in 2 1 2; do
  VIBA_GROUPS_V=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-banded-count > gpurun_out/bench_${T}_v$v.json 2> gpurun_out/bench_${T}_v$v.log || exit 1
  python -c "import json,sys; d=json.loads(open('gpurun_out/bench_${T}_v$v.json').read().strip().splitlines()[-1]); print('v$v', round(d['value'],2), d['phases_ms'])"
done
