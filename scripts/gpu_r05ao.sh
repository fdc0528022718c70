#!/bin/bash
# fan-in workgroups per level launch (VIBA_SN_FANWGS, divided among the active streams) re-swept
# on the two-stream schedule
set -o pipefail
mkdir -p gpurun_out
T=r05ao
for rep in 1 2 3; do
  for v in 3072 2048 4096 6144; do
    VIBA_SN_FANWGS=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-banded-count > gpurun_out/bench_${T}.json 2> gpurun_out/bench_${T}.log || { tail -20 gpurun_out/bench_${T}.log; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/bench_${T}.json').read().strip().splitlines()[-1]); print('fanwgs $v', round(d['value'],2), d['phases_ms']['factor_ms'])"
  done
done
