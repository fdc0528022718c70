#!/bin/bash
# bench config C under several environment settings (same library), one line each:
#   bash scripts/gpu_env_sweep.sh "" "VIBA_FAN_SORT=1" "VIBA_FANIN_WGS=4096 VIBA_FAN_SORT=1"
mkdir -p gpurun_out
i=0
for e in "$@"; do
  i=$((i + 1))
  env $e timeout -k 10 300 python bench.py --no-cpu-baseline --steps 4 --warmup 1 > gpurun_out/env_$i.json 2> gpurun_out/env_$i.log || exit $?
  echo "[$e]: $(grep timed gpurun_out/env_$i.log | sed 's/.*last it: //') | $(python -c "import json;j=json.load(open('gpurun_out/env_$i.json'));r=j['roofline'];print(round(j['value'],2),'it/s', round(r['achieved'],1),r['unit'])")"
done
