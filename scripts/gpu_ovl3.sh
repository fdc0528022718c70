#!/bin/bash
# potrf on a high-priority stream beside the off-diagonal fan-in: parity with the overlap on, then bench
# on / off (profiled and graphed)
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/ovl3
VIBA_POTRF_OVERLAP=1 timeout -k 10 900 python -u -m pytest tests/test_parity_gpu.py tests/test_parity_configs.py tests/test_distributed_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread > ${O}_pytest.log 2>&1; rc=$?; tail -3 ${O}_pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
for v in 0 1; do
VIBA_POTRF_OVERLAP=$v timeout -k 10 300 python bench.py --no-cpu-baseline > ${O}_$v$i.json 2>${O}_$v$i.log || exit $?
VIBA_POTRF_OVERLAP=$v timeout -k 10 300 python bench.py --no-cpu-baseline --profile-family -1 > ${O}_g$v$i.json 2>${O}_g$v$i.log || exit $?
python -c "import json;d=json.load(open('${O}_$v$i.json'));e=json.load(open('${O}_g$v$i.json'));print('overlap=$v', round(d['value'],2), round(d['roofline']['frac'],3), d['phases_ms']['factor_ms'], 'graphed', round(e['value'],2), e['phases_ms']['factor_ms'])"
done; done
