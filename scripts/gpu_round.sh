#!/bin/bash
# Round measurement: separate PMC passes (FETCH_SIZE, WRITE_SIZE) for the roofline traffic, summarised and
# stamped with the measured sources (and installed as this box's profiles/pmc_summary.json, so the bench
# line below reports its traffic as measured on these sources), then the default bench (with CPU
# baseline), then rocprofv3 kernel stats of the same command.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TAG=${1:-r01}
COMMIT=${2:-unknown}  # the commit of the measured sources (the box has no .git): stamped into the PMC summary
RE="fanin_kernel|visual_lin_kernel|schur_run[0-9]_kernel|landmark_|obs_group_kernel|trsm_kernel|potrf|small_assemble|zero_tiles"
cd /tmp
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$RE" --output-format csv -d $R/gpurun_out/pmc_fetch_$TAG -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-banded-count > /dev/null 2> $R/gpurun_out/pmc_fetch_$TAG.log || exit $?
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$RE" --output-format csv -d $R/gpurun_out/pmc_write_$TAG -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-banded-count > /dev/null 2> $R/gpurun_out/pmc_write_$TAG.log || exit $?
cd $R && python scripts/pmc_summary.py gpurun_out/pmc_fetch_$TAG gpurun_out/pmc_write_$TAG gpurun_out/pmc_summary_$TAG.json $COMMIT > /dev/null || exit $?
cp gpurun_out/pmc_summary_$TAG.json profiles/pmc_summary.json || exit $?
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.log || exit $?
cd /tmp
# (rocprofv3 traces the graph replays too since ROCm 7.2; the two-stream factorization launches eagerly)
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o run -- python3 $R/bench.py --no-cpu-baseline --no-banded-count > $R/gpurun_out/bench_${TAG}_prof.json 2> $R/gpurun_out/bench_${TAG}_prof.log || exit $?
