#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
export VIBA_NO_FUSE_POTRF=1
timeout -k 10 300 python bench.py --config C --steps 2 --warmup 1 --no-cpu-baseline --profile-family 3 > gpurun_out/nf.json 2> gpurun_out/nf.log; echo "rc=$?"
