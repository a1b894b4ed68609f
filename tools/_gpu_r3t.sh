set -o pipefail
mkdir -p gpurun_out/t
timeout -k 10 400 python -u -m pytest tests/test_gpu_node.py tests/test_gpu_configs.py tests/test_gpu_train.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t/test.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/t/test.log; [ $rc -eq 0 ] || exit $rc
VARIANTS="old main" ROUNDS=3 BENCH_ARGS="--node --config 3 --steps 10 --warmup 3 --no-seam" bash tools/ab_bench.sh || exit 1
VARIANTS="old main" ROUNDS=2 BENCH_ARGS="--force-collectives --config 3 --steps 10 --warmup 3 --no-seam" bash tools/ab_bench.sh || exit 1
