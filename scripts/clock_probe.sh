#!/bin/bash
# Shader / memory clocks read (rocm-smi, read-only) while the bench's LM loop runs, and once idle.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 60 rocm-smi --showclocks > gpurun_out/clk_idle.txt 2>&1 || true
timeout -k 10 400 python bench.py --steps 3000 --warmup 2 --no-cpu-baseline --no-banded-count > gpurun_out/clk_bench.json 2> gpurun_out/clk_bench.log &
pid=$!
sleep 25
for i in $(seq 1 12); do
  timeout -k 10 30 rocm-smi --showclocks >> gpurun_out/clk_busy.txt 2>&1 || true
  sleep 3
done
wait $pid
