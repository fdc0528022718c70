#!/bin/bash
# profiled factorization kept in its HIP graph (event-record nodes around the fan-in launches): parity,
# the bench with and without it, and the rocprof kernel averages to compare the event timing against
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/pg
timeout -k 10 900 python -u -m pytest tests/test_parity_gpu.py tests/test_parity_configs.py tests/test_covariances.py tests/test_abi.py tests/test_pcg.py -x -q -m gpu --timeout 300 --timeout-method thread > ${O}_pytest.log 2>&1; rc=$?; tail -3 ${O}_pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 300 python bench.py --no-cpu-baseline > ${O}_g$i.json 2>${O}_g$i.log || exit $?
VIBA_PROF_GRAPHS=0 timeout -k 10 300 python bench.py --no-cpu-baseline > ${O}_e$i.json 2>${O}_e$i.log || exit $?
done
for f in g1 e1 g2 e2; do python -c "import json;d=json.load(open('${O}_$f.json'));r=d['roofline'];print('$f', round(d['value'],2), 'frac', round(r['frac'],4), 'avg_ms', round(r['avg_launch_ms'],5), r['launches'], d['phases_ms']['factor_ms'])"; done
bash scripts/gpu_kstats.sh pg > ${O}_kstats.txt 2>&1 || exit $?
head -12 ${O}_kstats.txt
