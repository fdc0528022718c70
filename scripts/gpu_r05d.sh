#!/bin/bash
# supernode v3 (forward substitution inside the block loop): parity, profile, A/B
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_supernode_gpu.py -m gpu > gpurun_out/pytest_r05d.log 2>&1 || { tail -40 gpurun_out/pytest_r05d.log; exit 1; }
grep -h "passed\|failed" gpurun_out/pytest_r05d.log
TAG=r05d_sn
(cd /tmp && VIBA_SUPERNODE=1 VIBA_NO_GRAPHS=1 timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$TAG -o run -- python3 $R/bench.py --no-cpu-baseline --no-banded-count --steps 3 --warmup 1 > $R/gpurun_out/$TAG.json 2> $R/gpurun_out/$TAG.log) || exit $?
f=$(ls gpurun_out/$TAG/*kernel_trace.csv gpurun_out/$TAG/*/*kernel_trace.csv 2>/dev/null | head -1)
python scripts/level_profile.py $f > gpurun_out/${TAG}_levels.txt
tail -1 gpurun_out/${TAG}_levels.txt
python scripts/prof_summary.py $(dirname $f) 16 | grep -E "fanin|potrf|trsm|copy_diag|diag_inv"
for cfg in "0 x" "1 256" "1 512" "0 x" "1 256" "1 128"; do
  set -- $cfg
  VIBA_SUPERNODE=$1 VIBA_SN_FUSE=$2 timeout -k 10 300 python bench.py --no-cpu-baseline --no-banded-count --steps 20 --warmup 2 > gpurun_out/r05d_ab.json 2> gpurun_out/r05d_ab.log || exit $?
  python -c "import json;d=json.loads(open('gpurun_out/r05d_ab.json').read().strip().splitlines()[-1]);print('sn',$1,'fuse','$2',round(d['value'],2),d['phases_ms']['factor_ms'])"
done
