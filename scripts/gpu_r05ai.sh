#!/bin/bash
# more pairs of VIBA_SN_OFFSET 0 / 1 / 2 (r05ah was within noise)
set -o pipefail
mkdir -p gpurun_out
T=r05ai
for rep in 1 2 3 4; do
  for v in 0 1 2; do
    VIBA_SN_OFFSET=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-banded-count > gpurun_out/bench_${T}.json 2> gpurun_out/bench_${T}.log || { tail -20 gpurun_out/bench_${T}.log; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/bench_${T}.json').read().strip().splitlines()[-1]); print('offset $v', round(d['value'],2), d['phases_ms']['factor_ms'])"
  done
done
