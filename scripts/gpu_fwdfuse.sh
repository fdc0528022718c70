#!/bin/bash
# forward solve fused into the factorization: parity (factorization-dependent GPU tests), then the bench
# with and without it
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_parity_gpu.py tests/test_parity_configs.py tests/test_covariances.py tests/test_session_gpu.py tests/test_preint.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/fwdfuse_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/fwdfuse_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline 2>gpurun_out/fwdfuse_bench.log || exit $?
VIBA_FWD_IN_FACTOR=0 timeout -k 10 300 python bench.py --no-cpu-baseline 2>gpurun_out/fwdfuse_bench0.log
