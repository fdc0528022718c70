#!/bin/bash
# PCG path: GPU tests, then config C with each preconditioner (40 iterations, the reference default)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_pcg.py -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/pcg_t.log 2>&1 || { grep -E "PASS|FAIL|Error|assert" gpurun_out/pcg_t.log | head -30; exit 1; }
grep -c PASSED gpurun_out/pcg_t.log
for S in ${SOLVERS:-pcg-jacobi pcg-gauss-seidel}; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 --warmup 1 --solver $S > gpurun_out/pcg_$S.json 2> gpurun_out/pcg_$S.log || exit 1
  echo "$S: $(grep -h 'timed\|PCG' gpurun_out/pcg_$S.log)"
done
