#!/bin/bash
# potrf beside the off-diagonal fan-in: parity of the factorization-dependent GPU tests, then the bench
# with and without the overlap, profiled (ungraphed factorization) and unprofiled (graphs)
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/ovl
timeout -k 10 900 python -u -m pytest tests/test_parity_gpu.py tests/test_parity_configs.py tests/test_covariances.py tests/test_distributed_gpu.py tests/test_abi.py -x -q -m gpu --timeout 300 --timeout-method thread > ${O}_pytest.log 2>&1; rc=$?; tail -3 ${O}_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > ${O}_on.json 2>${O}_on.log || exit $?
VIBA_POTRF_OVERLAP=0 timeout -k 10 300 python bench.py --no-cpu-baseline > ${O}_off.json 2>${O}_off.log || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --profile-family -1 > ${O}_on_g.json 2>${O}_on_g.log || exit $?
VIBA_POTRF_OVERLAP=0 timeout -k 10 300 python bench.py --no-cpu-baseline --profile-family -1 > ${O}_off_g.json 2>${O}_off_g.log || exit $?
for f in on off on_g off_g; do python -c "import json;d=json.load(open('${O}_$f.json'));r=d.get('roofline') or {};print('$f', round(d['value'],2), r.get('frac'), d.get('phases_ms', ''))"; done
