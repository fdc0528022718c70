#!/bin/bash
# run selected -m gpu tests (pytest -k expression in $1), then optionally a bench: gpu_sel.sh "expr" [bench]
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-sel}
timeout -k 10 1000 python -u -m pytest tests/ -x -v -m gpu --timeout 600 --timeout-method thread -k "$1" -s > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
grep -E "PASSED|FAILED|config|miniB|passed|failed" gpurun_out/${TAG}_pytest.log | tail -30
if [ "$2" = "bench" ]; then
  timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.log || exit $?
  python -c "import json;d=json.load(open('gpurun_out/${TAG}_bench.json'));print(round(d['value'],2), d['phases_ms'])"
fi
