#!/bin/bash
# quick GPU check after a kernel change: the core parity tests, then one bench run (no CPU baseline)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-qc}
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_parity_gpu.py tests/test_parity_configs.py > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/${TAG}_pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.log || exit $?
grep timed gpurun_out/${TAG}_bench.log
exit $rc
