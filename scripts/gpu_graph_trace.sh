#!/bin/bash
# rocprofv3 kernel trace of the production path: the factorization replayed from its HIP graph
# (--profile-family -1: no per-launch events), short config-C run; records whether the tracer survives
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_graph -o run -- python3 $R/bench.py --no-cpu-baseline --profile-family -1 --steps 3 --warmup 1 > $R/gpurun_out/graph_trace.json 2> $R/gpurun_out/graph_trace.log
rc=$?
echo "rocprofv3 over the graphed factorization: rc=$rc"
tail -5 $R/gpurun_out/graph_trace.log
exit 0
