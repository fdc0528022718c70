#!/bin/bash
# bench.py's multi-process path on a one-GPU box: 2 ranks over gloo sharing cuda:0 (RCCL refuses two
# ranks on one device); partition mode (default for a power of two) and landmark shards
set -o pipefail
mkdir -p gpurun_out
export VIBA_DIST_BACKEND=gloo VIBA_DIST_SAME_DEVICE=1
for mode in partition shard; do
  VIBA_MULTI=$mode timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 ${EXTRA:-} > gpurun_out/dist_$mode.json 2> gpurun_out/dist_$mode.log || { tail -20 gpurun_out/dist_$mode.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/dist_$mode.json').read().strip().splitlines()[-1]);print('$mode', round(d['value'],2), d['n_gpus'], d['roofline']['frac'], d['roofline']['traffic'], (d['cpu_baseline'] or {}).get('value'))"
done
