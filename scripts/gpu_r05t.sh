#!/bin/bash
# experiment: unequal stream weights (VIBA_SN_SKEW = stream 0's share) to keep the two streams out of phase
set -o pipefail
mkdir -p gpurun_out
T=r05t
for k in none 0.6 0.7 none 0.6 0.7; do
  E=""; [ $k != none ] && E="VIBA_SN_SKEW=$k"
  env $E VIBA_FACTOR_STATS=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-banded-count > gpurun_out/bench_${T}.json 2> gpurun_out/bench_${T}.log || { tail -20 gpurun_out/bench_${T}.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/bench_${T}.json').read().strip().splitlines()[-1]); r=d['roofline']; print('skew $k', round(d['value'],2), d['phases_ms']['factor_ms'], 'frac', round(r['frac'],3))"
  grep "factor stats\] stream" gpurun_out/bench_${T}.log | head -2
done
