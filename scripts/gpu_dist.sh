#!/bin/bash
# sharded LM on one GPU: the GPU distributed test + bench.py's run_sharded with 2 ranks (gloo)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_distributed_gpu.py -x -q > gpurun_out/pytest_dist.log 2>&1; rc=$?
tail -30 gpurun_out/pytest_dist.log
[ $rc -eq 0 ] || exit $rc
export VIBA_DIST_BACKEND=gloo VIBA_DIST_SAME_DEVICE=1
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 2 --warmup 1 --config B > gpurun_out/bench_dist.json 2> gpurun_out/bench_dist.log; rc=$?
tail -5 gpurun_out/bench_dist.log; cat gpurun_out/bench_dist.json
exit $rc
