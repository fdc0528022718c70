#!/bin/bash
# GPU tests, default bench (no CPU baseline) and an eager kernel trace of config C; stops at the first
# failing step
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-chk}
timeout -k 10 400 python -u -m pytest tests/ -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_$TAG.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.log || { cat gpurun_out/bench_$TAG.log; exit 1; }
cat gpurun_out/bench_$TAG.log
python -c "import json; d=json.load(open('gpurun_out/bench_$TAG.json')); print('value', d['value'], 'ms', d['ms_per_step'], 'fanin', d['roofline']['achieved'])"
[ "${TRACE:-1}" = "1" ] && bash scripts/gpu_trace.sh trace_$TAG
exit 0
