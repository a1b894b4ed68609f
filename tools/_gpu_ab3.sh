set -o pipefail
VARIANTS="main multi" ROUNDS=2 BENCH_ARGS="--config 5 --steps 3 --warmup 1 --no-seam" bash tools/ab_bench.sh || exit 1
grep -h -o '"tslot": [0-9.]*' gpurun_out/ab/*.log
VARIANTS="main multi" ROUNDS=2 BENCH_ARGS="--steps 20 --warmup 5 --no-seam" bash tools/ab_bench.sh || exit 1
grep -h -o '"tslot": [0-9.]*' gpurun_out/ab/*.log
DBSCAN_LIB_PATH=dbscan-on-spark_amd/lib_ab/multi/libdbscan_hip.so timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_batch.py tests/test_gpu_node.py -m gpu -x -q --timeout 280 --timeout-method thread > gpurun_out/ab/multi_test.log 2>&1; echo "multi tests rc=$?"; tail -1 gpurun_out/ab/multi_test.log
