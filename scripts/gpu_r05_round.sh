#!/bin/bash
# round-5 measurement: the default bench line (CPU baseline included), its rocprofv3 kernel stats, separate
# FETCH_SIZE / WRITE_SIZE PMC passes, the config-E (mixed) line + its kernel stats, and the N = 2 / N = 8
# multi-process lines on this one GPU (gloo, ranks sharing cuda:0: the protocol and its phase split, not
# a scaling measurement)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TAG=${1:-r05f}
RE="fanin_kernel|visual_lin_kernel|schur_run[0-9]_kernel|landmark_obs|obs_group_kernel|trsm_kernel|potrf|small_assemble|zero_tiles"
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.log || exit $?
tail -1 gpurun_out/bench_$TAG.json | cut -c1-400
cd /tmp
(VIBA_NO_GRAPHS=1 timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o run -- python3 $R/bench.py --no-cpu-baseline --no-banded-count > $R/gpurun_out/bench_${TAG}_prof.json 2> $R/gpurun_out/bench_${TAG}_prof.log) || exit $?
(timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$RE" --output-format csv -d $R/gpurun_out/pmc_fetch_$TAG -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-banded-count > /dev/null 2> $R/gpurun_out/pmc_fetch_$TAG.log) || exit $?
(timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$RE" --output-format csv -d $R/gpurun_out/pmc_write_$TAG -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-banded-count > /dev/null 2> $R/gpurun_out/pmc_write_$TAG.log) || exit $?
cd $R
python scripts/pmc_summary.py gpurun_out/pmc_fetch_$TAG gpurun_out/pmc_write_$TAG gpurun_out/pmc_summary_$TAG.json > /dev/null || exit $?
f=$(ls gpurun_out/prof_$TAG/*kernel_stats.csv gpurun_out/prof_$TAG/*/*kernel_stats.csv 2>/dev/null | head -1)
python scripts/prof_summary.py $(dirname $f) 12
python scripts/busy_union.py $(dirname $f)/run_kernel_trace.csv fanin_kernel snpotrf sntrsm > gpurun_out/busy_union_$TAG.json || exit 1
python scripts/factor_overlap.py $(dirname $f)/run_kernel_trace.csv > gpurun_out/factor_overlap_$TAG.txt || exit 1
timeout -k 10 600 python bench.py --precision mixed --no-cpu-baseline > gpurun_out/bench_${TAG}_mixed.json 2> gpurun_out/bench_${TAG}_mixed.log || exit $?
tail -1 gpurun_out/bench_${TAG}_mixed.json | cut -c1-300
(cd /tmp && VIBA_NO_GRAPHS=1 timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_${TAG}_mixed -o run -- python3 $R/bench.py --precision mixed --no-cpu-baseline --no-banded-count > $R/gpurun_out/bench_${TAG}_mixed_prof.json 2> $R/gpurun_out/bench_${TAG}_mixed_prof.log) || exit $?
export VIBA_DIST_BACKEND=gloo VIBA_DIST_SAME_DEVICE=1
for N in 2 8; do
  timeout -k 10 900 python bench.py --gpus $N --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_${TAG}_n$N.json 2> gpurun_out/bench_${TAG}_n$N.log || { tail -20 gpurun_out/bench_${TAG}_n$N.log; exit 1; }
  tail -1 gpurun_out/bench_${TAG}_n$N.json | cut -c1-300
done
