#!/bin/bash
# stream count A/B on one box: 2 vs 3 streams, three runs each, interleaved
set -o pipefail
mkdir -p gpurun_out
T=r05s
for n in 2 3 2 3 2 3; do
  VIBA_SN_STREAMS=$n timeout -k 10 300 python bench.py --no-cpu-baseline --no-banded-count > gpurun_out/bench_${T}.json 2> gpurun_out/bench_${T}.log || { tail -20 gpurun_out/bench_${T}.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/bench_${T}.json').read().strip().splitlines()[-1]); r=d['roofline']; print('streams $n', round(d['value'],2), d['phases_ms']['factor_ms'], 'frac', round(r['frac'],3))"
done
