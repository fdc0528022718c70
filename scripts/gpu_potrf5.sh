#!/bin/bash
# 16x16 factor without redundant selects: micro, parity, bench x2
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/p5
timeout -k 10 120 python scripts/micro_potrf.py > ${O}_micro.log 2>&1 || exit $?; cat ${O}_micro.log
timeout -k 10 900 python -u -m pytest tests/test_parity_gpu.py tests/test_parity_configs.py tests/test_covariances.py tests/test_pcg.py tests/test_ordering_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread > ${O}_pytest.log 2>&1; rc=$?; tail -2 ${O}_pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do timeout -k 10 300 python bench.py --no-cpu-baseline > ${O}_$i.json 2>${O}_$i.log || exit $?
python -c "import json;d=json.load(open('${O}_$i.json'));print(round(d['value'],2), d['phases_ms']['factor_ms'])"; done
