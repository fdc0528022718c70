#!/bin/bash
# supernode schedule as the default: A/B (XCD-mapped row kernels), then the whole -m gpu suite
set -o pipefail
mkdir -p gpurun_out
for sn in 0 1 0 1; do
  VIBA_SUPERNODE=$sn timeout -k 10 300 python bench.py --no-cpu-baseline --no-banded-count --steps 20 --warmup 2 > gpurun_out/r05e_ab.json 2> gpurun_out/r05e_ab.log || exit $?
  python -c "import json;d=json.loads(open('gpurun_out/r05e_ab.json').read().strip().splitlines()[-1]);print('sn',$sn,round(d['value'],2),d['phases_ms']['factor_ms'])"
done
timeout -k 10 1700 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/pytest_r05e.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_r05e.log
exit $rc
