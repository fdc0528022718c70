#!/bin/bash
# the second factorization stream started one diagonal-block launch (1) or one level's rows (2) after the
# first (VIBA_SN_OFFSET), so their levels run out of phase
set -o pipefail
mkdir -p gpurun_out
T=r05ah
VIBA_SN_OFFSET=2 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_supernode_gpu.py > gpurun_out/pytest_${T}.log 2>&1 || { tail -30 gpurun_out/pytest_${T}.log; exit 1; }
tail -1 gpurun_out/pytest_${T}.log
for rep in 1 2; do
  for v in 0 1 2; do
    VIBA_SN_OFFSET=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-banded-count > gpurun_out/bench_${T}.json 2> gpurun_out/bench_${T}.log || { tail -20 gpurun_out/bench_${T}.log; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/bench_${T}.json').read().strip().splitlines()[-1]); print('offset $v', round(d['value'],2), round(d['roofline']['frac'],3), d['phases_ms']['factor_ms'])"
  done
done
