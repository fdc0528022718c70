#!/bin/bash
# Parameterised GPU-box launcher (replaces the per-variant gpu_rNN*.sh one-offs):
#   scripts/gpu_run.sh TAG pytest "<pytest -k expression or test path args>"
#   scripts/gpu_run.sh TAG bench "<bench.py args>"            (env knobs via VAR=value before the script)
#   scripts/gpu_run.sh TAG kstats "<bench.py args>"           (rocprofv3 --kernel-trace --stats of bench.py)
#   scripts/gpu_run.sh TAG pmc "<counter>" "<bench.py args>"  (one --pmc pass of bench.py)
# Output under gpurun_out/<TAG>_*; every GPU step under its own timeout; the first failure ends the run.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; WHAT=$2; shift 2
case "$WHAT" in
  pytest)
    timeout -k 10 ${T:-900} python -u -m pytest -x -v --timeout ${TT:-300} --timeout-method thread -m gpu $1 \
      > gpurun_out/${TAG}_pytest.log 2>&1 ;;
  bench)
    timeout -k 10 ${T:-600} python bench.py $1 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.log ;;
  kstats)
    cd /tmp && timeout -k 10 ${T:-600} rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_prof \
      -o run -- python3 $R/bench.py $1 > $R/gpurun_out/${TAG}_prof.json 2> $R/gpurun_out/${TAG}_prof.log ;;
  pmc)
    cd /tmp && timeout -s KILL ${T:-300} rocprofv3 --pmc $1 --output-format csv -d $R/gpurun_out/${TAG}_pmc_$1 -o run \
      -- python3 $R/bench.py $2 > /dev/null 2> $R/gpurun_out/${TAG}_pmc_$1.log ;;
  *) echo "unknown step $WHAT"; exit 2 ;;
esac
