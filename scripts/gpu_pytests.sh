#!/bin/bash
# run several pytest selections in sequence on the GPU box; stop at anything worse than a test failure
mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
for sel in "$@"; do
  i=$((i+1))
  timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu $sel > gpurun_out/pyt_$i.log 2>&1; rc=$?
  echo "== [$sel] rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed|Error" gpurun_out/pyt_$i.log | tail -25
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
