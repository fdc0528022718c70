#!/bin/bash
# linearize side streams (clear on its own stream): parity, bench x2, one-iteration timeline
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/side
timeout -k 10 900 python -u -m pytest tests/test_parity_gpu.py tests/test_parity_configs.py tests/test_distributed_gpu.py tests/test_covariances.py -x -q -m gpu --timeout 300 --timeout-method thread > ${O}_pytest.log 2>&1; rc=$?; tail -3 ${O}_pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do timeout -k 10 300 python bench.py --no-cpu-baseline > ${O}_$i.json 2>${O}_$i.log || exit $?
python -c "import json;d=json.load(open('${O}_$i.json'));print(round(d['value'],2), d['phases_ms'])"; done
bash scripts/gpu_trace.sh side_tr && python scripts/timeline.py $(ls gpurun_out/side_tr/*kernel_trace.csv | head -1) > ${O}_timeline.txt && head -22 ${O}_timeline.txt
