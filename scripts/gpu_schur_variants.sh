#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for k in 3 0; do
  VIBA_SCHUR=$k timeout -k 10 120 python -u -m pytest tests/test_parity_gpu.py -x -q -k "one_lm_step or optimize_trajectory" --timeout 100 --timeout-method thread > gpurun_out/schur_t$k.log 2>&1 || { echo "tests failed for $k"; tail -20 gpurun_out/schur_t$k.log; exit 1; }
  tail -1 gpurun_out/schur_t$k.log
  VIBA_SCHUR=$k timeout -k 10 200 python bench.py --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/schur_b$k.json 2> gpurun_out/schur_b$k.log || exit 1
  echo "VIBA_SCHUR=$k"; grep timed gpurun_out/schur_b$k.log
done
