#!/bin/bash
# GPU pass: the whole -m gpu suite (per-test timeout), smoke, one default bench run
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-pass}
timeout -k 10 1500 python -u -m pytest tests/ -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1; rc=$?
tail -60 gpurun_out/${TAG}_pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.log; rc2=$?
tail -5 gpurun_out/${TAG}_bench.log; cat gpurun_out/${TAG}_bench.json
exit $rc
