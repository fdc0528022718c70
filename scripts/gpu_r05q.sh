#!/bin/bash
# the round's bench line with the refreshed PMC summary (profiles/pmc_summary.json from r05p)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python bench.py > gpurun_out/bench_r05q.json 2> gpurun_out/bench_r05q.log || { tail -20 gpurun_out/bench_r05q.log; exit 1; }
tail -1 gpurun_out/bench_r05q.json | cut -c1-300
