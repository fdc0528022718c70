#!/bin/bash
# list the PMC counters of this device, then run PMC groups over kernels matching $1 (gpu_pmc_kernel.sh)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $GRAFT_REPO_ROOT/gpurun_out/counters_list.txt 2>&1 || true
cd $GRAFT_REPO_ROOT
bash scripts/gpu_pmc_kernel.sh "$@" > gpurun_out/pmck_summary.txt 2>&1 || { tail -20 gpurun_out/pmck_summary.txt; exit 1; }
cat gpurun_out/pmck_summary.txt
