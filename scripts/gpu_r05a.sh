#!/bin/bash
# round-5 first check: the new and changed tests first, then the whole -m gpu suite, then the default bench
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -v -s --timeout 600 --timeout-method thread"
timeout -k 10 900 $T tests/test_lm_controller.py tests/test_optimize_gpu.py tests/test_session_gpu.py \
  "tests/test_parity_gpu.py::test_one_lm_step_matches_oracle" -m gpu > gpurun_out/pytest_r05a_new.log 2>&1 || { tail -30 gpurun_out/pytest_r05a_new.log; exit 1; }
grep -h "gradient entry errors" gpurun_out/pytest_r05a_new.log || true
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench_r05a.json 2> gpurun_out/bench_r05a.log || exit $?
timeout -k 10 1200 $T tests/test_distributed_gpu.py -m gpu -k "eight or bench" > gpurun_out/pytest_r05a_dist.log 2>&1 || { tail -30 gpurun_out/pytest_r05a_dist.log; exit 1; }
tail -3 gpurun_out/pytest_r05a_dist.log
