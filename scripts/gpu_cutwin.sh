#!/bin/bash
# nested-dissection cut window / separator side: contributions, levels, it/s
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/cw
for v in "0 0" "0.1 0" "0.25 0" "0.1 1" "0.25 1"; do set -- $v
VIBA_ND_CUTWIN=$1 VIBA_ND_SEPRIGHT=$2 timeout -k 10 300 python bench.py --no-cpu-baseline > ${O}_$1_$2.json 2>${O}_$1_$2.log || exit $?
grep "finalize" ${O}_$1_$2.log | sed "s/^/w=$1 r=$2 /" | cut -c1-200
python -c "import json;d=json.load(open('${O}_$1_$2.json'));print('w=$1 r=$2', round(d['value'],2), d['phases_ms']['factor_ms'], d['phases_ms']['schur_ms'], d['phases_ms']['solve_ms'])"
done
