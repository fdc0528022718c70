#!/bin/bash
# four-wave potrf: single-tile launch times of the three forms, parity of the factorization-dependent GPU
# tests on the default form, then the bench on each form
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/potrf4
for v in "VIBA_POTRF_WAVES=1" "VIBA_DIAG_INV=lds" "VIBA_DIAG_INV=dpp"; do
  env $v timeout -k 10 120 python scripts/micro_potrf.py >> ${O}_micro.log 2>&1 || exit $?
done
cat ${O}_micro.log
timeout -k 10 900 python -u -m pytest tests/test_parity_gpu.py tests/test_parity_configs.py tests/test_covariances.py tests/test_abi.py -x -q -m gpu --timeout 300 --timeout-method thread > ${O}_pytest.log 2>&1; rc=$?; tail -3 ${O}_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > ${O}_bench_dpp.json 2>${O}_bench_dpp.log || exit $?
VIBA_DIAG_INV=lds timeout -k 10 300 python bench.py --no-cpu-baseline > ${O}_bench_lds.json 2>${O}_bench_lds.log || exit $?
VIBA_POTRF_WAVES=1 timeout -k 10 300 python bench.py --no-cpu-baseline > ${O}_bench_w1.json 2>${O}_bench_w1.log || exit $?
for f in dpp lds w1; do python -c "import json;d=json.load(open('${O}_bench_$f.json'));print('$f', d['value'], d.get('phases_ms', ''))"; done
