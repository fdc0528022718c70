#!/bin/bash
# round-4 final measurement: bench + rocprof stats + PMC, the small-factor kernel probe, smoke, full -m gpu suite
set -o pipefail
bash scripts/gpu_round.sh r04x || exit $?
timeout -k 10 200 python scripts/kernel_probe.py C 5 fp64 0,1,2,10,12,13,14,15,16,17,18,19 > gpurun_out/kp_r04x.json 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r04x.log 2>&1 || exit $?
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r04x.log 2>&1
tail -2 gpurun_out/pytest_r04x.log
