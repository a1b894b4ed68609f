bash tools/gpu_node_check.sh || exit $?
timeout -k 10 120 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --steps 3 --warmup 1 --points-per-gpu 2000000 > gpurun_out/bench_nccl2.log 2>&1
echo "nccl2 rc=$?"; grep '^{' gpurun_out/bench_nccl2.log | cut -c1-600; grep -iE "error|duplicate" gpurun_out/bench_nccl2.log | head -5
exit 0
