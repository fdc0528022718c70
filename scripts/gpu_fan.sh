#!/bin/bash
# fan-in variants: bench each library build, print factor ms and the fan-in's average launch
set -o pipefail
mkdir -p gpurun_out
for L in "$@"; do
  VIBA_LIB_DIR=$GRAFT_REPO_ROOT/visual_inertial_bundle_adjustment_amd/$L timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/fan_$L.json 2> gpurun_out/fan_$L.log || { tail -5 gpurun_out/fan_$L.log; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/fan_$L.json'));r=d['roofline'];print('$L', round(d['value'],2), d['phases_ms']['factor_ms'], round(r['avg_launch_ms']*1e3,1), round(r['achieved'],1))"
done
