#!/bin/bash
# fan-in experiment (scripts/fan_expt.py) over SPEC = libdir[:VAR=v,VAR2=w] (environment switches per run)
set -o pipefail
mkdir -p gpurun_out
i=0
for spec in "$@"; do
  lib=${spec%%:*}; envs=""
  [ "$spec" != "$lib" ] && envs=${spec#*:}
  env VIBA_LIB_DIR=$GRAFT_REPO_ROOT/visual_inertial_bundle_adjustment_amd/$lib ${envs//,/ } timeout -k 10 300 python scripts/fan_expt.py > gpurun_out/fxe_$i.json 2> gpurun_out/fxe_$i.log || { tail -5 gpurun_out/fxe_$i.log; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/fxe_$i.json'));print('$spec', [round(x[1],3) for x in d['launches_ms']])"
  i=$((i+1))
done
