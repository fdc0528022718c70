#!/bin/bash
# scripts/schur_probe.py against several library builds: gpu_probe.sh libdir[:VAR=v] ...
set -o pipefail
mkdir -p gpurun_out
for spec in "$@"; do
  lib=${spec%%:*}; envs=""
  [ "$spec" != "$lib" ] && envs=${spec#*:}
  env VIBA_LIB_DIR=$GRAFT_REPO_ROOT/visual_inertial_bundle_adjustment_amd/$lib ${envs//,/ } timeout -k 10 300 python scripts/schur_probe.py 2> gpurun_out/probe_$lib.log || { tail -5 gpurun_out/probe_$lib.log; exit 1; }
done
