#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/potrf4_timing.log
for L in lib_timing lib_timing3; do
  echo "== $L" >> gpurun_out/potrf4_timing.log
  VIBA_LIB_DIR=$PWD/visual_inertial_bundle_adjustment_amd/$L timeout -k 10 120 python scripts/micro_potrf4_timing.py >> gpurun_out/potrf4_timing.log 2>&1 || exit $?
done
cat gpurun_out/potrf4_timing.log
