#!/bin/bash
# three factorization streams against two on the current tree (the spare-store clear on stF at G = 3)
set -o pipefail
mkdir -p gpurun_out
T=r05af
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_supernode_gpu.py tests/test_lm_controller.py > gpurun_out/pytest_${T}.log 2>&1 \
  || { tail -30 gpurun_out/pytest_${T}.log; exit 1; }
tail -3 gpurun_out/pytest_${T}.log
for v in 3 2 3 2 3 2; do
  VIBA_SN_STREAMS=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-banded-count > gpurun_out/bench_${T}.json 2> gpurun_out/bench_${T}.log || { tail -20 gpurun_out/bench_${T}.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/bench_${T}.json').read().strip().splitlines()[-1]); print('streams $v', round(d['value'],2), round(d['roofline']['frac'],3), d['phases_ms'])"
done
