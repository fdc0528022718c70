#!/bin/bash
# kernel + memory-copy trace of the default bench's timed loop (the profiled fan-in family runs eagerly,
# as in the bench line), then the device idle between kernels (scripts/gaps.py)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TAG=${1:-gaps}
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $R/gpurun_out/$TAG -o run -- python3 $R/bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-banded-count > $R/gpurun_out/$TAG.json 2> $R/gpurun_out/$TAG.log || exit $?
cd $R && python scripts/gaps.py $(find gpurun_out/$TAG -name '*kernel_trace.csv' | head -1) 3 16 > gpurun_out/${TAG}_gaps.txt
