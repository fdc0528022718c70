#!/bin/bash
# the whole -m gpu suite, then two default bench runs (profiled fan-in) and one unprofiled
set -o pipefail
mkdir -p gpurun_out
T=${1:-full}
timeout -k 10 1500 python -u -m pytest tests/ -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1; rc=$?
tail -5 gpurun_out/${T}_pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/${T}_b$i.json 2>gpurun_out/${T}_b$i.log || exit $?; done
timeout -k 10 300 python bench.py --no-cpu-baseline --profile-family -1 > gpurun_out/${T}_n.json 2>gpurun_out/${T}_n.log || exit $?
for f in b1 b2 n; do python -c "import json;d=json.load(open('gpurun_out/${T}_$f.json'));r=d['roofline'] or {};print('$f', round(d['value'],2), r.get('frac'), d['phases_ms'])"; done
