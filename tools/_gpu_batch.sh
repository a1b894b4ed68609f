set -o pipefail
mkdir -p gpurun_out/b
timeout -k 10 600 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_small.py -m gpu --maxfail=5 -v --timeout 300 --timeout-method thread > gpurun_out/b/test.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -8 gpurun_out/b/test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --seam-only --no-cpu-baseline > gpurun_out/b/seam.log 2>&1
rc=$?; echo "seam rc=$rc"; tail -c 3000 gpurun_out/b/seam.log; exit $rc
