#!/bin/bash
# A/B knobs: Schur item order (VIBA_SCHUR_ORDER), row kernel occupancy (VIBA_SN_TRSM_W4)
set -o pipefail
mkdir -p gpurun_out
run() {
  env $1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-banded-count --steps 20 --warmup 2 > gpurun_out/r05h_ab.json 2> gpurun_out/r05h_ab.log || exit $?
  python -c "import json;d=json.loads(open('gpurun_out/r05h_ab.json').read().strip().splitlines()[-1]);p=d['phases_ms'];print('$1',round(d['value'],2),'schur',p['schur_ms'],'factor',p['factor_ms'])"
}
for i in 1 2; do
  run VIBA_X=0
  run VIBA_SCHUR_ORDER=1
  run VIBA_SN_TRSM_W4=1
done
