#!/bin/bash
# the speculative rolling-shutter rebuild beside the cost pass: speculation / session parity, bench A/B
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
T=r05x
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_optimize_gpu.py tests/test_lm_controller.py tests/test_session_gpu.py tests/test_parity_configs.py > gpurun_out/pytest_$T.log 2>&1 || { tail -30 gpurun_out/pytest_$T.log; exit 1; }
tail -2 gpurun_out/pytest_$T.log
for v in new old new old; do
  L=""; [ $v = old ] && L="VIBA_LIB_DIR=$R/build_ab/old"
  env $L timeout -k 10 300 python bench.py --no-cpu-baseline --no-banded-count > gpurun_out/bench_${T}.json 2> gpurun_out/bench_${T}.log || { tail -20 gpurun_out/bench_${T}.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/bench_${T}.json').read().strip().splitlines()[-1]); print('$v', round(d['value'],2), d['phases_ms'])"
done
