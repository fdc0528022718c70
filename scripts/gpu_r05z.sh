#!/bin/bash
# experiment: main stream at high priority, side streams low (VIBA_STREAM_PRIO)
set -o pipefail
mkdir -p gpurun_out
T=r05z
for v in 1 0 1 0; do
  VIBA_STREAM_PRIO=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-banded-count > gpurun_out/bench_${T}.json 2> gpurun_out/bench_${T}.log || { tail -20 gpurun_out/bench_${T}.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/bench_${T}.json').read().strip().splitlines()[-1]); print('prio $v', round(d['value'],2), d['phases_ms'])"
done
