#!/bin/bash
# rocprofv3 kernel stats of the graphed bench for several library builds (args: libdirs); prints the
# fan-in / potrf / trsm / schur kernels' average durations per build
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for L in "$@"; do
  cd /tmp
  VIBA_LIB_DIR=$R/visual_inertial_bundle_adjustment_amd/$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/kab_$L -o run -- python3 $R/bench.py --no-cpu-baseline --profile-family -1 --steps 5 --warmup 2 > $R/gpurun_out/kab_$L.json 2> $R/gpurun_out/kab_$L.log || { tail -5 $R/gpurun_out/kab_$L.log; exit 1; }
  cd $R
  echo "== $L"
  python scripts/prof_summary.py gpurun_out/kab_$L 8
done
