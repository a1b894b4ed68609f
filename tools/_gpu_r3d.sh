set -o pipefail
mkdir -p gpurun_out/d
run() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > gpurun_out/d/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; tail -3 gpurun_out/d/$name.log; [ $rc -eq 0 ] || exit $rc
}
run bucket 700 python -u -m pytest tests/test_gpu_bucket.py tests/test_gpu_configs.py -m gpu -x -v --timeout 600 --timeout-method thread
run c4 200 python bench.py --config 4 --steps 5 --warmup 2 --no-cpu-baseline --e2e-steps 0 --no-seam
run c5 200 python bench.py --config 5 --steps 5 --warmup 2 --no-cpu-baseline --e2e-steps 0 --no-seam
grep -h '^{' gpurun_out/d/c4.log gpurun_out/d/c5.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['ms_per_step'], list(d['kernels_ms_per_step'].items())[:12])"
VARIANTS="main b20" ROUNDS=2 BENCH_ARGS="--steps 20 --warmup 5 --no-seam" timeout -k 10 400 bash tools/ab_bench.sh > gpurun_out/d/ab_c2.log 2>&1; echo "ab c2 rc=$?"; cat gpurun_out/d/ab_c2.log
VARIANTS="main b20" ROUNDS=2 BENCH_ARGS="--config 3 --steps 20 --warmup 5 --no-seam" timeout -k 10 400 bash tools/ab_bench.sh > gpurun_out/d/ab_c3.log 2>&1; echo "ab c3 rc=$?"; cat gpurun_out/d/ab_c3.log
