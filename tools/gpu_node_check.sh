#!/bin/bash
# Node path on the 1-GPU box: HIP slab kernels + real collectives (gloo; RCCL needs a GPU
# per rank), then bench.py through torch.distributed.run with 2 ranks on the one GPU.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_gpu_node.py -x -q --timeout 800 > gpurun_out/gpu_node_tests.log 2>&1
rc=$?; echo "node tests rc=$rc"; tail -3 gpurun_out/gpu_node_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --backend gloo --points-per-gpu 5000000 > gpurun_out/bench_node2.log 2>&1
rc=$?; echo "bench node rc=$rc"; grep '^{' gpurun_out/bench_node2.log | tail -1 | cut -c1-900
[ $rc -eq 0 ] || { tail -30 gpurun_out/bench_node2.log; exit $rc; }
timeout -k 10 300 python bench.py --node --steps 5 --warmup 2 > gpurun_out/bench_node1.log 2>&1
rc=$?; echo "bench node1 rc=$rc"; grep '^{' gpurun_out/bench_node1.log | tail -1 | cut -c1-900
exit $rc
