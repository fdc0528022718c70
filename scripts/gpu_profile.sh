#!/bin/bash
# one GPU session: bench at config B and C with kernel-family timing, plus rocprofv3 stats of config B
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --config C --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/benchC.json 2> gpurun_out/benchC.log || exit $?
timeout -k 10 300 python bench.py --config C --steps 3 --warmup 1 --no-cpu-baseline --profile-family 0 > gpurun_out/benchC_vis.json 2> gpurun_out/benchC_vis.log || exit $?
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_B -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config B --steps 2 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/benchB_prof.json 2> $GRAFT_REPO_ROOT/gpurun_out/benchB_prof.log
