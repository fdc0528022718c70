#!/bin/bash
# multi-rank LM on one GPU: the GPU distributed tests + bench.py's N>1 path (gloo, ranks sharing the
# device: a functional rehearsal, not a scaling measurement) in both multi-device modes
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
CFG=${1:-B}
timeout -k 10 600 python -m pytest tests/test_distributed_gpu.py -x -q > gpurun_out/pytest_dist.log 2>&1; rc=$?
tail -30 gpurun_out/pytest_dist.log
[ $rc -eq 0 ] || exit $rc
export VIBA_DIST_BACKEND=gloo VIBA_DIST_SAME_DEVICE=1
for m in partition shard; do
  VIBA_MULTI=$m timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 --config $CFG > gpurun_out/bench_dist_$m.json 2> gpurun_out/bench_dist_$m.log; rc=$?
  tail -5 gpurun_out/bench_dist_$m.log; cat gpurun_out/bench_dist_$m.json
  [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 600 python bench.py --steps 3 --warmup 1 --config $CFG > gpurun_out/bench_1.json 2> gpurun_out/bench_1.log; rc=$?
cat gpurun_out/bench_1.json
exit $rc
