#!/bin/bash
# rocprofv3 kernel stats of a short default bench (graphs off: the profiled family runs eagerly anyway)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TAG=${1:-ks}
cd /tmp
export VIBA_NO_GRAPHS=1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o run -- python3 $R/bench.py --no-cpu-baseline --steps 3 --warmup 1 > $R/gpurun_out/bench_${TAG}_prof.json 2> $R/gpurun_out/bench_${TAG}_prof.log || exit $?
cd $R && python scripts/prof_summary.py gpurun_out/prof_$TAG 24
