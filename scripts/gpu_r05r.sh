#!/bin/bash
# full -m gpu suite + smoke on the committed tree
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_r05r.log 2>&1 || { tail -40 gpurun_out/pytest_r05r.log; exit 1; }
tail -3 gpurun_out/pytest_r05r.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r05r.log 2>&1 || { tail -20 gpurun_out/smoke_r05r.log; exit 1; }
tail -3 gpurun_out/smoke_r05r.log
