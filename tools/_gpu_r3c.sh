set -o pipefail
mkdir -p gpurun_out/c
run() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > gpurun_out/c/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; tail -4 gpurun_out/c/$name.log; [ $rc -eq 0 ] || exit $rc
}
run batch 400 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_small.py -m gpu -x -v --timeout 300 --timeout-method thread
run bucket 700 python -u -m pytest tests/test_gpu_bucket.py tests/test_gpu_configs.py -m gpu -x -v --timeout 600 --timeout-method thread
run seam 300 python bench.py --seam-only --no-cpu-baseline
run c4 200 python bench.py --config 4 --steps 5 --warmup 2 --no-cpu-baseline --e2e-steps 0 --no-seam
run c5 200 python bench.py --config 5 --steps 5 --warmup 2 --no-cpu-baseline --e2e-steps 0 --no-seam
grep -h '^{' gpurun_out/c/c4.log gpurun_out/c/c5.log | cut -c1-300
