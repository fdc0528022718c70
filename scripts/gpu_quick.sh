#!/bin/bash
# quick loop: GPU parity tests + bench C + rocprof kernel stats (graphs off)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests/test_parity_gpu.py -x -q > gpurun_out/quick_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/quick_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/quick_bench.json 2> gpurun_out/quick_bench.log || exit $?
grep timed gpurun_out/quick_bench.log
cd /tmp && export VIBA_NO_GRAPHS=1 && timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_quick -o run -- python3 $R/bench.py --no-cpu-baseline --steps 3 --warmup 1 > /dev/null 2> $R/gpurun_out/quick_prof.log
