set -o pipefail
mkdir -p gpurun_out/fin3
VARIANTS="old main" ROUNDS=2 BENCH_ARGS="--config 5 --steps 3 --warmup 1 --no-seam" bash tools/ab_bench.sh || exit 1
grep -h -o '"tslot": [0-9.]*' gpurun_out/ab/*.log
VARIANTS="old main" ROUNDS=2 BENCH_ARGS="--steps 20 --warmup 5 --no-seam" bash tools/ab_bench.sh || exit 1
grep -h -o '"tslot": [0-9.]*' gpurun_out/ab/*.log
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/fin3/gputest.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/fin3/gputest.log; [ $rc -eq 0 ] || exit $rc
TAG=round3_q bash tools/round_evidence.sh
