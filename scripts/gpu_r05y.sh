#!/bin/bash
# single-launch variable backup / restore: optimize (restore paths) + distributed parity, bench, trace
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=r05y
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_optimize_gpu.py tests/test_lm_controller.py tests/test_parity_gpu.py tests/test_distributed_gpu.py > gpurun_out/pytest_$T.log 2>&1 || { tail -30 gpurun_out/pytest_$T.log; exit 1; }
tail -2 gpurun_out/pytest_$T.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-banded-count > gpurun_out/bench_${T}.json 2> gpurun_out/bench_${T}.log || { tail -20 gpurun_out/bench_${T}.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/bench_${T}.json').read().strip().splitlines()[-1]); print(round(d['value'],2), d['phases_ms'])"
done
cd /tmp
(timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_$T -o run -- python3 $R/bench.py --no-cpu-baseline --no-banded-count --profile-family -1 > /dev/null 2> $R/gpurun_out/prof_$T.log) || exit 1
cd $R
python scripts/timeline.py gpurun_out/prof_$T/run_kernel_trace.csv | grep -v "snpotrf\|sntrsm\|fanin"
