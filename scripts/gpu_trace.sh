#!/bin/bash
# kernel trace of config C (eager launches: rocprofv3 tracing crashes on hipGraph replays) for
# scripts/level_profile.py / timeline.py
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp VIBA_NO_GRAPHS=1
R=$GRAFT_REPO_ROOT
TAG=${1:-trace}
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$TAG -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/$TAG.json 2> $R/gpurun_out/$TAG.log
