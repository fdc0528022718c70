#!/bin/bash
# potrf + trsm fused for the levels with few off-diagonal tiles: parity, then the bench over the threshold
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/ptf
timeout -k 10 900 python -u -m pytest tests/test_parity_gpu.py tests/test_parity_configs.py tests/test_covariances.py tests/test_distributed_gpu.py tests/test_session_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread > ${O}_pytest.log 2>&1; rc=$?; tail -3 ${O}_pytest.log; [ $rc -eq 0 ] || exit $rc
for v in 0 256 64 1024 100000; do
VIBA_PT_FUSE=$v timeout -k 10 300 python bench.py --no-cpu-baseline > ${O}_$v.json 2>${O}_$v.log || exit $?
python -c "import json;d=json.load(open('${O}_$v.json'));r=d['roofline'] or {};print('fuse<=$v', round(d['value'],2), r.get('frac'), d['phases_ms']['factor_ms'], d['phases_ms']['solve_ms'])"
done
