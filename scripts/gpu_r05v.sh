#!/bin/bash
# wide landmarks beside the narrow class (VIBA_LANDMARK_SIDE) + 24-record group chunks: parity, bench A/B
set -o pipefail
mkdir -p gpurun_out
T=r05v
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_parity_gpu.py tests/test_optimize_gpu.py tests/test_session_gpu.py > gpurun_out/pytest_$T.log 2>&1 || { tail -30 gpurun_out/pytest_$T.log; exit 1; }
tail -2 gpurun_out/pytest_$T.log
for v in 1 0 1 0; do
  VIBA_LANDMARK_SIDE=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-banded-count > gpurun_out/bench_${T}.json 2> gpurun_out/bench_${T}.log || { tail -20 gpurun_out/bench_${T}.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/bench_${T}.json').read().strip().splitlines()[-1]); print('side $v', round(d['value'],2), d['phases_ms'])"
done
