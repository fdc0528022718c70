#!/bin/bash
# column vs supernode factorization: kernel stats + per-level profile of each; the bench-line test
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for SN in 0 1; do
  TAG=r05b_sn$SN
  (cd /tmp && VIBA_SUPERNODE=$SN VIBA_NO_GRAPHS=1 timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$TAG -o run -- python3 $R/bench.py --no-cpu-baseline --no-banded-count --steps 3 --warmup 1 > $R/gpurun_out/$TAG.json 2> $R/gpurun_out/$TAG.log) || exit $?
  f=$(ls gpurun_out/$TAG/*kernel_trace.csv gpurun_out/$TAG/*/*kernel_trace.csv 2>/dev/null | head -1)
  python scripts/level_profile.py $f > gpurun_out/${TAG}_levels.txt
  tail -2 gpurun_out/${TAG}_levels.txt
  d=$(dirname $f)
  python scripts/prof_summary.py $d 14
done
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread tests/test_distributed_gpu.py -k bench -m gpu > gpurun_out/pytest_r05b.log 2>&1 || { tail -30 gpurun_out/pytest_r05b.log; exit 1; }
tail -2 gpurun_out/pytest_r05b.log
