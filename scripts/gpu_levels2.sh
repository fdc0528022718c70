#!/bin/bash
# per-level factorization profile without and with the fused potrf + trsm levels
set -o pipefail
mkdir -p gpurun_out
VIBA_PT_FUSE=0 bash scripts/gpu_levels.sh lv0 > /dev/null || exit $?
bash scripts/gpu_levels.sh lv1 > /dev/null || exit $?
tail -3 gpurun_out/lv0_levels.txt; tail -3 gpurun_out/lv1_levels.txt
