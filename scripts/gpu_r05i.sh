#!/bin/bash
# solo kernel times of the linearize / Schur kernels on config C (vb_bench_kernel)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python scripts/kernel_probe.py C 5 fp64 10,12,13,14,15 > gpurun_out/probe_r05i.json 2> gpurun_out/probe_r05i.log || { tail -5 gpurun_out/probe_r05i.log; exit 1; }
cat gpurun_out/probe_r05i.json
