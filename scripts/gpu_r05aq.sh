#!/bin/bash
# look-ahead on the top separators' chain (VIBA_SN_LOOKAHEAD): a chain level's contributions from two or
# more levels down run on stF beside the previous level's diagonal block and rows
set -o pipefail
mkdir -p gpurun_out
T=r05aq
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_supernode_gpu.py tests/test_optimize_gpu.py tests/test_parity_gpu.py > gpurun_out/pytest_${T}.log 2>&1 \
  || { tail -30 gpurun_out/pytest_${T}.log; exit 1; }
tail -1 gpurun_out/pytest_${T}.log
for rep in 1 2 3; do
  for v in 1 0; do
    VIBA_SN_LOOKAHEAD=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-banded-count > gpurun_out/bench_${T}.json 2> gpurun_out/bench_${T}.log || { tail -20 gpurun_out/bench_${T}.log; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/bench_${T}.json').read().strip().splitlines()[-1]); r=d['roofline']; print('lookahead $v', round(d['value'],2), d['phases_ms']['factor_ms'], round(r['frac'],3))"
  done
done
