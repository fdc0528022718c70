#!/bin/bash
# cost pass beside the speculative linearization: optimize parity tests, bench, kernel trace timeline
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=r05n
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_optimize_gpu.py tests/test_lm_controller.py tests/test_supernode_gpu.py > gpurun_out/pytest_$T.log 2>&1 || { tail -30 gpurun_out/pytest_$T.log; exit 1; }
tail -2 gpurun_out/pytest_$T.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-banded-count > gpurun_out/bench_${T}_$i.json 2> gpurun_out/bench_${T}_$i.log || { tail -20 gpurun_out/bench_${T}_$i.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/bench_${T}_$i.json').read().strip().splitlines()[-1]); print(round(d['value'],2), d['phases_ms'])"
done
cd /tmp
(timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_$T -o run -- python3 $R/bench.py --no-cpu-baseline --no-banded-count --profile-family -1 > $R/gpurun_out/bench_${T}_prof.json 2> $R/gpurun_out/bench_${T}_prof.log) || exit $?
cd $R
python scripts/timeline.py gpurun_out/prof_$T/run_kernel_trace.csv | grep -v "snpotrf\\|sntrsm\\|fanin"
