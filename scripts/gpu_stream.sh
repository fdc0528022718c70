#!/bin/bash
# streamed fan-in: parity subset with the default and the split-K build, then the bench A/B
set -o pipefail
mkdir -p gpurun_out
K="one_lm_step or fused_factor or config_B_full or config_C_slice or full_size_properties or optimize_trajectory"
VIBA_FAN_STREAM=768 timeout -k 10 400 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread -k "$K" > gpurun_out/st_pytest0.log 2>&1 || { tail -30 gpurun_out/st_pytest0.log; exit 1; }
tail -1 gpurun_out/st_pytest0.log
VIBA_LIB_DIR=$GRAFT_REPO_ROOT/visual_inertial_bundle_adjustment_amd/lib_m4a VIBA_FAN_STREAM=512 timeout -k 10 400 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread -k "$K" > gpurun_out/st_pytest1.log 2>&1 || { tail -30 gpurun_out/st_pytest1.log; exit 1; }
tail -1 gpurun_out/st_pytest1.log
bash scripts/gpu_ab.sh st "$@"
