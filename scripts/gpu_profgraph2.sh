#!/bin/bash
# kernel start/stop events inside the captured graph (VIBA_PROF_GRAPHS=2) against eager profiling and
# an unprofiled graph
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/pg2
for i in 1 2; do
VIBA_PROF_GRAPHS=2 timeout -k 10 300 python bench.py --no-cpu-baseline > ${O}_x$i.json 2>${O}_x$i.log || exit $?
VIBA_PROF_GRAPHS=0 timeout -k 10 300 python bench.py --no-cpu-baseline > ${O}_e$i.json 2>${O}_e$i.log || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --profile-family -1 > ${O}_n$i.json 2>${O}_n$i.log || exit $?
done
for f in x1 e1 n1 x2 e2 n2; do python -c "import json;d=json.load(open('${O}_$f.json'));r=d['roofline'] or {};print('$f', round(d['value'],2), 'frac', r.get('frac'), 'avg_ms', r.get('avg_launch_ms'), r.get('launches'), d['phases_ms']['factor_ms'])"; done
