#!/bin/bash
# bench the same workload against alternative in-tree library builds (VIBA_LIB_DIR=...); args: lib dirs
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for L in "$@"; do
  VIBA_LIB_DIR=$GRAFT_REPO_ROOT/visual_inertial_bundle_adjustment_amd/$L timeout -k 10 200 python bench.py --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/sweep_$L.json 2> gpurun_out/sweep_$L.log || exit 1
  echo "$L: $(grep timed gpurun_out/sweep_$L.log)"
done
