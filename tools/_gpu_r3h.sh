set -o pipefail
mkdir -p gpurun_out/h
timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_node.py tests/test_gpu_bucket.py tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/h/gputest.log 2>&1
rc=$?; echo "gputest rc=$rc"; tail -4 gpurun_out/h/gputest.log; exit $rc
