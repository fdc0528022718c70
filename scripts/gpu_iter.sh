#!/bin/bash
# parity smoke + config-C bench (kernel families: gemm, schur) + rocprofv3 kernel stats on config C
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python scripts/gpu_first.py > gpurun_out/parity.log 2>&1 || { echo parity failed; exit 1; }
timeout -k 10 400 python bench.py --config C --steps 3 --warmup 1 --no-cpu-baseline --profile-family 4 > gpurun_out/benchC.json 2> gpurun_out/benchC.log || exit $?
timeout -k 10 400 python bench.py --config C --steps 3 --warmup 1 --no-cpu-baseline --profile-family 2 > gpurun_out/benchC_schur.json 2> gpurun_out/benchC_schur.log || exit $?
cd /tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_C -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config C --steps 2 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/benchC_prof.json 2> $GRAFT_REPO_ROOT/gpurun_out/benchC_prof.log
