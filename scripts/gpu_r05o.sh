#!/bin/bash
# cost pass beside the speculative linearization + paired Schur gathers: parity, Schur A/B, bench A/B
set -o pipefail
mkdir -p gpurun_out
T=r05o
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_parity_gpu.py tests/test_parity_configs.py tests/test_optimize_gpu.py tests/test_lm_controller.py > gpurun_out/pytest_$T.log 2>&1 || { tail -30 gpurun_out/pytest_$T.log; exit 1; }
tail -2 gpurun_out/pytest_$T.log
for v in pair nopair; do
  L=""; [ $v = nopair ] && L="VIBA_LIB_DIR=$GRAFT_REPO_ROOT/build_ab/nopair"
  env $L timeout -k 10 300 python scripts/kernel_probe.py C 5 fp64,mixed 14 > gpurun_out/probe_${T}_$v.json 2> gpurun_out/probe_${T}_$v.log || { tail -5 gpurun_out/probe_${T}_$v.log; exit 1; }
  echo $v $(python -c "import json; d=json.load(open('gpurun_out/probe_${T}_$v.json')); print({k: v['Schur tile products'] for k, v in d.items()})")
done
for v in pair nopair pair nopair; do
  L=""; [ $v = nopair ] && L="VIBA_LIB_DIR=$GRAFT_REPO_ROOT/build_ab/nopair"
  env $L timeout -k 10 300 python bench.py --no-cpu-baseline --no-banded-count > gpurun_out/bench_${T}_$v.json 2> gpurun_out/bench_${T}_$v.log || { tail -20 gpurun_out/bench_${T}_$v.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/bench_${T}_$v.json').read().strip().splitlines()[-1]); print('$v', round(d['value'],2), d['phases_ms'])"
done
