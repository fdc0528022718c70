#!/bin/bash
# Schur tile products: gathers two steps ahead (altlib1: all tasks, 3 waves / SIMD; altlib2: tasks of <= 4
# MFMA blocks, 4 waves / SIMD) against one step ahead (the default build); parity on each, then A/B
set -o pipefail
mkdir -p gpurun_out
T=r05ag
R=$GRAFT_REPO_ROOT
for L in altlib1 altlib2; do
  VIBA_LIB_DIR=$R/$L timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_parity_gpu.py > gpurun_out/pytest_${T}_$L.log 2>&1 || { tail -30 gpurun_out/pytest_${T}_$L.log; exit 1; }
  echo "$L: $(tail -1 gpurun_out/pytest_${T}_$L.log)"
done
for rep in 1 2; do
  for L in lib altlib1 altlib2; do
    if [ $L = lib ]; then D=$R/visual_inertial_bundle_adjustment_amd/lib; else D=$R/$L; fi
    VIBA_LIB_DIR=$D timeout -k 10 300 python bench.py --no-cpu-baseline --no-banded-count > gpurun_out/bench_${T}.json 2> gpurun_out/bench_${T}.log || { tail -20 gpurun_out/bench_${T}.log; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/bench_${T}.json').read().strip().splitlines()[-1]); print('$L', round(d['value'],2), d['phases_ms']['schur_ms'], d['phases_ms']['factor_ms'])"
  done
done
