#!/bin/bash
# r02e: parity (factorization + distributed) after the prefetching trsm and the engine-stream RCCL
# ordering, one default bench, then a 2-rank run of the multi-GPU bench on one GPU (RCCL probe)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r02e}
timeout -k 10 900 python -u -m pytest tests/test_parity_gpu.py tests/test_parity_configs.py tests/test_distributed_gpu.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { tail -30 gpurun_out/${T}_pytest.log; exit 1; }
tail -3 gpurun_out/${T}_pytest.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.log || exit $?
cat gpurun_out/${T}_bench.json
VIBA_DIST_SAME_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --config B --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_dist_nccl.json 2> gpurun_out/${T}_dist_nccl.log; echo "nccl rc=$?"
tail -5 gpurun_out/${T}_dist_nccl.log; cat gpurun_out/${T}_dist_nccl.json
