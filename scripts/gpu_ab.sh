#!/bin/bash
# A/B bench of the in-tree build against alternative library builds (VIBA_LIB_DIR); optional GPU
# parity tests first (set TESTS=1).  args: lib dirs under visual_inertial_bundle_adjustment_amd/
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
  timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_pytest.log 2>&1 || { tail -30 gpurun_out/ab_pytest.log; exit 1; }
  tail -2 gpurun_out/ab_pytest.log
fi
for L in lib "$@" lib; do
  VIBA_LIB_DIR=$GRAFT_REPO_ROOT/visual_inertial_bundle_adjustment_amd/$L timeout -k 10 200 python bench.py --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/ab_$L.json 2> gpurun_out/ab_$L.log || exit 1
  echo "$L: $(grep timed gpurun_out/ab_$L.log)"
done
