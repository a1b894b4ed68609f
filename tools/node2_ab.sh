#!/bin/bash
# Two ranks on the one GPU (gloo): the node step with and without the roots' gather stream.
set -o pipefail
mkdir -p gpurun_out
for v in 1 0 1 0; do
  DBSCAN_NODE_COMM_STREAM=$v timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --backend gloo --steps 10 --warmup 3 > gpurun_out/b2_$v.log 2>&1 || exit 1
  echo "comm_stream=$v $(grep -h '^{' gpurun_out/b2_$v.log | python -c 'import json,sys; print(json.loads(sys.stdin.readline())["ms_per_step"])')"
done
