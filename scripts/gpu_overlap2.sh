#!/bin/bash
# graphed factorization (nothing profiled): overlap on / off
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/ovl
for i in 1 2; do
timeout -k 10 300 python bench.py --no-cpu-baseline --profile-family -1 > ${O}_on_g$i.json 2>${O}_on_g$i.log || exit $?
VIBA_POTRF_OVERLAP=0 timeout -k 10 300 python bench.py --no-cpu-baseline --profile-family -1 > ${O}_off_g$i.json 2>${O}_off_g$i.log || exit $?
VIBA_POTRF_OVERLAP=0 timeout -k 10 300 python bench.py --no-cpu-baseline > ${O}_off_p$i.json 2>${O}_off_p$i.log || exit $?
done
for f in on_g1 off_g1 off_p1 on_g2 off_g2 off_p2; do python -c "import json;d=json.load(open('${O}_$f.json'));print('$f', round(d['value'],2), d.get('phases_ms', ''))"; done
