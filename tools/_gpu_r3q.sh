set -o pipefail
mkdir -p gpurun_out/q
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/q/test.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/q/test.log; [ $rc -eq 0 ] || exit $rc
VARIANTS="old main" ROUNDS=2 BENCH_ARGS="--config 5 --steps 3 --warmup 1 --no-seam" bash tools/ab_bench.sh || exit 1
VARIANTS="old main" ROUNDS=2 BENCH_ARGS="--config 3 --steps 10 --warmup 3 --no-seam" bash tools/ab_bench.sh || exit 1
VARIANTS="old main" ROUNDS=2 BENCH_ARGS="--steps 20 --warmup 5 --no-seam" bash tools/ab_bench.sh || exit 1
