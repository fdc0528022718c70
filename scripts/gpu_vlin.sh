#!/bin/bash
# visual kernels without the scratch-resident projection Jacobian: parity, bench x2, kernel stats
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/vlin
timeout -k 10 900 python -u -m pytest tests/test_parity_gpu.py tests/test_parity_configs.py tests/test_session_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread > ${O}_pytest.log 2>&1; rc=$?; tail -3 ${O}_pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do timeout -k 10 300 python bench.py --no-cpu-baseline > ${O}_$i.json 2>${O}_$i.log || exit $?
python -c "import json;d=json.load(open('${O}_$i.json'));print(round(d['value'],2), d['phases_ms'])"; done
timeout -k 10 300 python bench.py --no-cpu-baseline --profile-family 0 > ${O}_p0.json 2>${O}_p0.log || exit $?
python -c "import json;d=json.load(open('${O}_p0.json'));r=d['roofline'];print('visual_lin', round(r['avg_launch_ms'],4), 'ms', round(r['achieved']), 'GB/s')"
