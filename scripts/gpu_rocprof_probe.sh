#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
export VIBA_NO_GRAPHS=1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/probe_nograph -o run -- python3 $R/bench.py --no-cpu-baseline > $R/gpurun_out/probe_nograph.json 2> $R/gpurun_out/probe_nograph.log; echo "nograph rc=$?"
