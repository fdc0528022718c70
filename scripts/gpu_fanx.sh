#!/bin/bash
# fan-in memory experiment over library builds: scripts/fan_expt.py per lib (args: libdirs)
set -o pipefail
mkdir -p gpurun_out
for L in "$@"; do
  VIBA_LIB_DIR=$GRAFT_REPO_ROOT/visual_inertial_bundle_adjustment_amd/$L timeout -k 10 300 python scripts/fan_expt.py > gpurun_out/fanx_$L.json 2> gpurun_out/fanx_$L.log || { tail -5 gpurun_out/fanx_$L.log; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/fanx_$L.json'));print('$L', [round(x[1],3) for x in d['launches_ms']], [round(t,1) for t in d['tflops']])"
done
