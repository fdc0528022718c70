#!/bin/bash
# per-kernel device time (rocprofv3 kernel stats) of the bench for alternative library builds; args: lib dirs
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp VIBA_NO_GRAPHS=1
R=$GRAFT_REPO_ROOT
for L in "$@"; do
  cd /tmp && VIBA_LIB_DIR=$R/visual_inertial_bundle_adjustment_amd/$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/lt_$L -o run -- python3 $R/bench.py --no-cpu-baseline --steps 3 --warmup 1 > /dev/null 2> $R/gpurun_out/lt_$L.log || exit 1
  echo "== $L"; head -12 $R/gpurun_out/lt_$L/run_kernel_stats.csv | cut -d, -f1-4 | sed 's/(viba::Dev[^"]*//'
done
