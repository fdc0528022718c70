#!/bin/bash
# nested-dissection cut window x separator side x leaf size
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/cw2
for v in "0.02 1 1024" "0.03 1 1024" "0.04 1 1024" "0.07 1 1024" "0.03 1 512" "0.05 1 512" "0.05 1 768" "0.03 1 768"; do set -- $v
VIBA_ND_CUTWIN=$1 VIBA_ND_SEPRIGHT=$2 VIBA_ND_LEAF=$3 timeout -k 10 300 python bench.py --no-cpu-baseline > ${O}_$1_$2_$3.json 2>${O}_$1_$2_$3.log || exit $?
pairs=$(grep -o "gemm pairs/factorization [0-9]*" ${O}_$1_$2_$3.log | awk '{print $3}'); lv=$(grep -o "[0-9]* levels" ${O}_$1_$2_$3.log)
python -c "import json;d=json.load(open('${O}_$1_$2_$3.json'));print('w=$1 r=$2 leaf=$3 pairs=$pairs $lv', round(d['value'],2), d['phases_ms']['factor_ms'], d['phases_ms']['solve_ms'])"
done
