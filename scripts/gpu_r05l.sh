#!/bin/bash
# supernode streams with cross-stream separator dependencies: parity, stream balance, bench A/B
set -o pipefail
mkdir -p gpurun_out
T=r05l
for c in B C; do
  VIBA_SCHUR_STATS=0 VIBA_SN_STREAMS=4 timeout -k 10 300 python scripts/symbolic_stats.py $c > gpurun_out/sym_${T}_$c.log 2>&1 || { tail -5 gpurun_out/sym_${T}_$c.log; exit 1; }
  grep "\[factor stats\] stream" gpurun_out/sym_${T}_$c.log
done
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_supernode_gpu.py tests/test_optimize_gpu.py > gpurun_out/pytest_$T.log 2>&1 || { tail -30 gpurun_out/pytest_$T.log; exit 1; }
tail -2 gpurun_out/pytest_$T.log
for n in 1 2 3 4 2; do
  VIBA_SN_STREAMS=$n timeout -k 10 300 python bench.py --no-cpu-baseline --no-banded-count > gpurun_out/bench_${T}_s$n.json 2> gpurun_out/bench_${T}_s$n.log || { tail -20 gpurun_out/bench_${T}_s$n.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/bench_${T}_s$n.json').read().strip().splitlines()[-1]); r=d['roofline']; print('streams $n', round(d['value'],2), d['phases_ms']['factor_ms'], d['phases_ms']['total_ms'], 'fanin avg', round(r['avg_launch_ms'],4), 'frac', round(r['frac'],3), 'launches/factor', r['fanin_launches_per_factorization'])"
done
