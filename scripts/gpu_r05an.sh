#!/bin/bash
# fused-level threshold (VIBA_SN_FUSE: levels with at most this many row items per active stream run
# snpotrf_trsm8) re-swept on the two-stream schedule
set -o pipefail
mkdir -p gpurun_out
T=r05an
for rep in 1 2 3; do
  for v in 256 128 512 1024; do
    VIBA_SN_FUSE=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-banded-count > gpurun_out/bench_${T}.json 2> gpurun_out/bench_${T}.log || { tail -20 gpurun_out/bench_${T}.log; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/bench_${T}.json').read().strip().splitlines()[-1]); print('fuse $v', round(d['value'],2), d['phases_ms']['factor_ms'])"
  done
done
