#!/bin/bash
# diagonal-tile inverses with split sums: parity, kernel time (rocprof), bench A/B against the previous build
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=r05w
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_parity_gpu.py tests/test_supernode_gpu.py tests/test_covariances.py > gpurun_out/pytest_$T.log 2>&1 || { tail -30 gpurun_out/pytest_$T.log; exit 1; }
tail -2 gpurun_out/pytest_$T.log
for v in new old; do
  cd /tmp
  if [ $v = old ]; then export VIBA_LIB_DIR=$R/build_ab/old; fi
  (timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_${T}_$v -o run -- python3 $R/bench.py --no-cpu-baseline --no-banded-count --steps 3 > /dev/null 2> $R/gpurun_out/prof_${T}_$v.log) || exit 1
  cd $R
  echo $v $(grep diag_inverse gpurun_out/prof_${T}_$v/run_kernel_stats.csv | cut -d, -f1-4)
done
unset VIBA_LIB_DIR
for v in new old new old; do
  L=""; [ $v = old ] && L="VIBA_LIB_DIR=$R/build_ab/old"
  env $L timeout -k 10 300 python bench.py --no-cpu-baseline --no-banded-count > gpurun_out/bench_${T}.json 2> gpurun_out/bench_${T}.log || { tail -20 gpurun_out/bench_${T}.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/bench_${T}.json').read().strip().splitlines()[-1]); print('$v', round(d['value'],2), d['phases_ms']['factor_ms'], d['phases_ms']['solve_ms'])"
done
