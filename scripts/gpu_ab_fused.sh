#!/bin/bash
# A/B of the fused factor level (factor_level_kernel) against the 3-launch level, + parity tests
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-fz}
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_parity_gpu.py tests/test_parity_configs.py tests/test_distributed_gpu.py -k "one_lm_step or trajectory or config_B or config_C or partitioned" > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -3 gpurun_out/${TAG}_pytest.log
for f in 1 0; do
  VIBA_FUSED_FACTOR=$f timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 > gpurun_out/${TAG}_bench_f$f.json 2> gpurun_out/${TAG}_bench_f$f.log || exit $?
  tail -1 gpurun_out/${TAG}_bench_f$f.log
  python -c "import json;d=json.load(open('gpurun_out/${TAG}_bench_f$f.json'));print('fused=$f', round(d['value'],2), d['phases_ms'])"
done
