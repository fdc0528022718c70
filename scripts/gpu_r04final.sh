#!/bin/bash
# round-4 closing check of the committed tree: smoke, the default bench line, the full -m gpu suite
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r04final.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > gpurun_out/bench_r04final.json 2> gpurun_out/bench_r04final.log || exit $?
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r04final.log 2>&1
tail -2 gpurun_out/pytest_r04final.log
