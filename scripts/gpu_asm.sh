#!/bin/bash
# small-factor assembly split over two streams: parity, bench x3
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/asm
timeout -k 10 900 python -u -m pytest tests/test_parity_gpu.py tests/test_parity_configs.py tests/test_covariances.py -x -q -m gpu --timeout 300 --timeout-method thread > ${O}_pytest.log 2>&1; rc=$?; tail -2 ${O}_pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do timeout -k 10 300 python bench.py --no-cpu-baseline > ${O}_$i.json 2>${O}_$i.log || exit $?
python -c "import json;d=json.load(open('${O}_$i.json'));print(round(d['value'],2), d['phases_ms'])"; done
