set -o pipefail
mkdir -p gpurun_out/u
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/u/test.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/u/test.log; [ $rc -eq 0 ] || exit $rc
VARIANTS="old main" ROUNDS=2 BENCH_ARGS="--config 4 --steps 5 --warmup 2 --no-seam" bash tools/ab_bench.sh || exit 1
grep -h -o '"big_count": [0-9.]*' gpurun_out/ab/*.log
VARIANTS="old main" ROUNDS=2 BENCH_ARGS="--steps 20 --warmup 5 --no-seam" bash tools/ab_bench.sh || exit 1
grep -h -o '"big_count": [0-9.]*' gpurun_out/ab/*.log
