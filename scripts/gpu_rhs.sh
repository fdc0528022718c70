#!/bin/bash
# new-RHS pass with register sums: parity (sub-step paths, shards), kernel stats of the bench
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/rhs
timeout -k 10 900 python -u -m pytest tests/test_parity_gpu.py tests/test_parity_configs.py tests/test_distributed_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread > ${O}_pytest.log 2>&1; rc=$?; tail -2 ${O}_pytest.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_kstats.sh rhs > ${O}_kstats.txt 2>&1 || exit $?
grep -E "reduced_rhs|fanin" ${O}_kstats.txt; python -c "import json;d=json.load(open('gpurun_out/bench_rhs_prof.json'));print(round(d['value'],2))"
