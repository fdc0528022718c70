#!/bin/bash
# re-tune after the ordering change: fused potrf+trsm threshold, fan-in workgroups per level
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/tn
for v in "256 3072" "512 3072" "256 4096" "512 4096" "256 6144" "512 6144" "256 8192" "512 2048"; do set -- $v
VIBA_PT_FUSE=$1 VIBA_FANIN_WGS=$2 timeout -k 10 300 python bench.py --no-cpu-baseline > ${O}_$1_$2.json 2>${O}_$1_$2.log || exit $?
python -c "import json;d=json.load(open('${O}_$1_$2.json'));print('fuse=$1 wgs=$2', round(d['value'],2), round(d['roofline']['frac'],4), d['phases_ms']['factor_ms'])"
done
