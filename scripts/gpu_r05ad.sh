#!/bin/bash
# the scalar read polls the readback stream instead of blocking (VIBA_SPIN_READ):
# controller parity tests, then a same-box A/B
set -o pipefail
mkdir -p gpurun_out
T=r05ad
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_optimize_gpu.py tests/test_parity_configs.py tests/test_lm_controller.py tests/test_supernode_gpu.py > gpurun_out/pytest_${T}.log 2>&1 \
  || { tail -30 gpurun_out/pytest_${T}.log; exit 1; }
tail -3 gpurun_out/pytest_${T}.log
for v in 1 0 1 0; do
  VIBA_SPIN_READ=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-banded-count > gpurun_out/bench_${T}.json 2> gpurun_out/bench_${T}.log || { tail -20 gpurun_out/bench_${T}.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/bench_${T}.json').read().strip().splitlines()[-1]); print('spin-read $v', round(d['value'],2), d['phases_ms'])"
done
