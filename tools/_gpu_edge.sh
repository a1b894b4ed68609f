set -o pipefail
mkdir -p gpurun_out/ed
VARIANTS="old main" ROUNDS=3 BENCH_ARGS="--steps 20 --warmup 5 --no-seam" bash tools/ab_bench.sh || exit 1
grep -h -o '"edge_union": [0-9.]*' gpurun_out/ab/*.log
VARIANTS="old main" ROUNDS=2 BENCH_ARGS="--config 3 --steps 10 --warmup 3 --no-seam" bash tools/ab_bench.sh || exit 1
grep -h -o '"edge_union": [0-9.]*' gpurun_out/ab/*.log
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ed/test.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/ed/test.log; exit $rc
