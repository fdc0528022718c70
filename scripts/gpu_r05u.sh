#!/bin/bash
# observation-group chunk size sweep (VIBA_GRP_CHUNK builds in build_ab/): the group kernel alone
set -o pipefail
mkdir -p gpurun_out
for c in 32 16 24 48 64 32; do
  L=""; [ $c != 32 ] && L="VIBA_LIB_DIR=$GRAFT_REPO_ROOT/build_ab/g$c"
  env $L timeout -k 10 300 python scripts/kernel_probe.py C 5 fp64,mixed 13 > gpurun_out/probe_r05u.json 2> gpurun_out/probe_r05u.log || { tail -5 gpurun_out/probe_r05u.log; exit 1; }
  echo chunk $c $(python -c "import json; d=json.load(open('gpurun_out/probe_r05u.json')); print({k: v['observation-group Gram blocks'] for k, v in d.items()})")
done
