#!/bin/bash
# A/B of library builds and environment switches on the default bench (config C, no CPU baseline):
#   gpu_ab.sh TAG [--test "pytest -k expr"] SPEC...   SPEC = libdir[:VAR=v,VAR2=w]  (libdir under the package)
# stops at the first failing step
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; shift
if [ "$1" = "--test" ]; then
  timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread -k "$2" > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
  tail -1 gpurun_out/${TAG}_pytest.log
  shift 2
fi
i=0
for spec in "$@"; do
  lib=${spec%%:*}; envs=""
  [ "$spec" != "$lib" ] && envs=${spec#*:}
  env VIBA_LIB_DIR=$GRAFT_REPO_ROOT/visual_inertial_bundle_adjustment_amd/$lib ${envs//,/ } timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/${TAG}_b$i.json 2> gpurun_out/${TAG}_b$i.log || { tail -5 gpurun_out/${TAG}_b$i.log; exit 1; }
  echo "$spec: $(python -c "import json;d=json.load(open('gpurun_out/${TAG}_b$i.json'));p=d['phases_ms'];print(round(d['value'],2), {k: p[k] for k in ('linearize_ms','schur_ms','factor_ms','solve_ms','cost_ms')})")"
  i=$((i+1))
done
