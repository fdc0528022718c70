#!/bin/bash
# fan-in by target pairs of two-column supernodes (VIBA_FAN_PAIRS): parity, then A/B
set -o pipefail
mkdir -p gpurun_out
T=r05aj
VIBA_FACTOR_STATS=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_supernode_gpu.py > gpurun_out/pytest_${T}.log 2>&1 || { tail -40 gpurun_out/pytest_${T}.log; exit 1; }
tail -1 gpurun_out/pytest_${T}.log
grep "fan-in items" gpurun_out/pytest_${T}.log | tail -2
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_parity_gpu.py tests/test_optimize_gpu.py tests/test_parity_configs.py > gpurun_out/pytest2_${T}.log 2>&1 || { tail -40 gpurun_out/pytest2_${T}.log; exit 1; }
tail -1 gpurun_out/pytest2_${T}.log
for rep in 1 2 3; do
  for v in 1 0; do
    VIBA_FAN_PAIRS=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-banded-count > gpurun_out/bench_${T}.json 2> gpurun_out/bench_${T}.log || { tail -20 gpurun_out/bench_${T}.log; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/bench_${T}.json').read().strip().splitlines()[-1]); r=d['roofline']; print('pairs $v', round(d['value'],2), d['phases_ms']['factor_ms'], round(r['busy_ms_per_factorization'],3), round(r['avg_launch_ms']*1000,1))"
  done
done
