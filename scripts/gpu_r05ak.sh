#!/bin/bash
# target-pair fan-in: ring 3 (default build) vs ring 2 (altlib1, 3 blocks / CU) vs single targets
set -o pipefail
mkdir -p gpurun_out
T=r05ak
R=$GRAFT_REPO_ROOT
VIBA_FACTOR_STATS=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-banded-count --steps 1 --warmup 0 > /dev/null 2> gpurun_out/stats_${T}.log || { tail -20 gpurun_out/stats_${T}.log; exit 1; }
grep "fan-in items" gpurun_out/stats_${T}.log | head -2
VIBA_LIB_DIR=$R/altlib1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_supernode_gpu.py > gpurun_out/pytest_${T}.log 2>&1 || { tail -40 gpurun_out/pytest_${T}.log; exit 1; }
tail -1 gpurun_out/pytest_${T}.log
for rep in 1 2; do
  for v in ring3 ring2 single; do
    D=$R/visual_inertial_bundle_adjustment_amd/lib; P=1
    [ $v = ring2 ] && D=$R/altlib1
    [ $v = single ] && P=0
    VIBA_LIB_DIR=$D VIBA_FAN_PAIRS=$P timeout -k 10 300 python bench.py --no-cpu-baseline --no-banded-count > gpurun_out/bench_${T}.json 2> gpurun_out/bench_${T}.log || { tail -20 gpurun_out/bench_${T}.log; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/bench_${T}.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$v', round(d['value'],2), d['phases_ms']['factor_ms'], round(r['busy_ms_per_factorization'],3), round(r['avg_launch_ms']*1000,1))"
  done
done
