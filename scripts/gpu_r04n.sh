#!/bin/bash
# round-4 closing batch: round measurement (bench + rocprof stats + PMC), landmark class-threshold probe,
# full -m gpu suite
set -o pipefail
R=$GRAFT_REPO_ROOT
bash scripts/gpu_round.sh r04n || exit $?
for v in lib lib_lm192 lib_lm384; do
  VIBA_LIB_DIR=$R/visual_inertial_bundle_adjustment_amd/$v timeout -k 10 150 python scripts/kernel_probe.py C 5 fp64 12 > gpurun_out/kp_$v.json 2>&1 || exit $?
done
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r04n.log 2>&1
tail -2 gpurun_out/pytest_r04n.log
