#!/bin/bash
# supernode rows staged in LDS (sntrsm_lds_kernel): parity, level profile, A/B against one block per row
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_supernode_gpu.py tests/test_parity_gpu.py -m gpu > gpurun_out/pytest_r05g.log 2>&1 || { tail -40 gpurun_out/pytest_r05g.log; exit 1; }
grep -h "passed\|failed" gpurun_out/pytest_r05g.log
TAG=r05g_sn
(cd /tmp && VIBA_NO_GRAPHS=1 timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$TAG -o run -- python3 $R/bench.py --no-cpu-baseline --no-banded-count --steps 3 --warmup 1 > $R/gpurun_out/$TAG.json 2> $R/gpurun_out/$TAG.log) || exit $?
f=$(ls gpurun_out/$TAG/*kernel_trace.csv gpurun_out/$TAG/*/*kernel_trace.csv 2>/dev/null | head -1)
python scripts/level_profile.py $f > gpurun_out/${TAG}_levels.txt
tail -1 gpurun_out/${TAG}_levels.txt
python scripts/prof_summary.py $(dirname $f) 18 | grep -E "fanin|potrf|trsm|copy_diag|diag_inv"
for cfg in "0 256" "1 256" "1 512" "0 256" "1 256" "1 128"; do
  set -- $cfg
  VIBA_SN_LDS=$1 VIBA_SN_BLOCKS=$2 timeout -k 10 300 python bench.py --no-cpu-baseline --no-banded-count --steps 20 --warmup 2 > gpurun_out/r05g_ab.json 2> gpurun_out/r05g_ab.log || exit $?
  python -c "import json;d=json.loads(open('gpurun_out/r05g_ab.json').read().strip().splitlines()[-1]);print('lds',$1,'blocks',$2,round(d['value'],2),d['phases_ms']['factor_ms'])"
done
timeout -k 10 1000 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_distributed_gpu.py -m gpu > gpurun_out/pytest_r05g_dist.log 2>&1 || { tail -40 gpurun_out/pytest_r05g_dist.log; exit 1; }
tail -2 gpurun_out/pytest_r05g_dist.log
