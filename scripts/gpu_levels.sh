#!/bin/bash
# kernel trace of config C + the per-level factorization profile (scripts/level_profile.py)
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-levels}
bash scripts/gpu_trace.sh $TAG || exit $?
f=$(ls gpurun_out/$TAG/*kernel_trace.csv gpurun_out/$TAG/*/*kernel_trace.csv 2>/dev/null | head -1)
python scripts/level_profile.py $f > gpurun_out/${TAG}_levels.txt
tail -30 gpurun_out/${TAG}_levels.txt
