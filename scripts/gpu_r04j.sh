#!/bin/bash
# round-4 batch: profiled-event harvest check, obs_group unroll A/B (kernel probe), rocprof stats of the
# bench (fan-in average against the event-timed one)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
VIBA_PROF_DEBUG=1 timeout -k 10 200 python scripts/prof_debug.py > gpurun_out/profdbg2.log 2>&1 || exit $?
timeout -k 10 150 python scripts/kernel_probe.py C 5 fp64 12,13 > gpurun_out/kp_u4.json 2>&1 || exit $?
VIBA_LIB_DIR=$R/visual_inertial_bundle_adjustment_amd/lib_u8 timeout -k 10 150 python scripts/kernel_probe.py C 5 fp64 12,13 > gpurun_out/kp_u8.json 2>&1 || exit $?
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/stats_r04j -o run -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-banded-count > $R/gpurun_out/bench_r04j_prof.json 2> $R/gpurun_out/bench_r04j_prof.log || exit $?
