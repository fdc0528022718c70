#!/bin/bash
# A/B of an environment switch on the default bench: gpu_ab_env.sh TAG "VAR=a" "VAR=b" [...]
# (runs the whole -m gpu suite first; stops at the first failing step)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; shift
timeout -k 10 900 python -u -m pytest tests/ -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest.log
i=0
for kv in "$@"; do
  env $kv timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/${TAG}_b$i.json 2> gpurun_out/${TAG}_b$i.log || exit $?
  echo "$kv: $(python -c "import json;d=json.load(open('gpurun_out/${TAG}_b$i.json'));print(round(d['value'],2), d['phases_ms'])")"
  i=$((i+1))
done
