set -o pipefail
mkdir -p gpurun_out/m
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --deselect tests/test_gpu_configs.py::test_config5_full_size_train_node > gpurun_out/m/test.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/m/test.log; [ $rc -eq 0 ] || exit $rc
VARIANTS="old halo main" ROUNDS=2 BENCH_ARGS="--config 5 --steps 3 --warmup 1 --no-seam" bash tools/ab_bench.sh || exit 1
mkdir -p gpurun_out/m/c5; cp gpurun_out/ab/*.log gpurun_out/m/c5/
VARIANTS="old halo main" ROUNDS=2 BENCH_ARGS="--steps 20 --warmup 5 --no-seam" bash tools/ab_bench.sh || exit 1
bash tools/profile.sh
