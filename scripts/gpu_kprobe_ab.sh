#!/bin/bash
# kernel_probe over several library builds: gpu_kprobe_ab.sh TAG KERNELS libdir...  (libdir under the package)
set -o pipefail
mkdir -p gpurun_out
TAG=$1 K=$2; shift 2
for lib in "$@"; do
  VIBA_LIB_DIR=$GRAFT_REPO_ROOT/visual_inertial_bundle_adjustment_amd/$lib timeout -k 10 200 python scripts/kernel_probe.py C 5 fp64 $K > gpurun_out/${TAG}_$lib.json 2>&1 || { tail -5 gpurun_out/${TAG}_$lib.json; exit 1; }
  echo "$lib: $(python -c "import json;print(json.load(open('gpurun_out/${TAG}_$lib.json'))['fp64'])")"
done
