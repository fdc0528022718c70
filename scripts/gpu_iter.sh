#!/bin/bash
# parity smoke + config-C bench + rocprofv3 kernel stats on config C (fused and unfused potrf)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python scripts/gpu_first.py > gpurun_out/parity.log 2>&1 || { echo parity failed; exit 1; }
timeout -k 10 400 python bench.py --config C --steps 3 --warmup 1 --no-cpu-baseline --profile-family 4 > gpurun_out/benchC.json 2> gpurun_out/benchC.log || exit $?
cd /tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_C -o run -- python3 $R/bench.py --config C --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/benchC_prof.json 2> $R/gpurun_out/benchC_prof.log || exit $?
export VIBA_NO_FUSE_POTRF=1
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_C_nofuse -o run -- python3 $R/bench.py --config C --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/benchC_prof2.json 2> $R/gpurun_out/benchC_prof2.log
