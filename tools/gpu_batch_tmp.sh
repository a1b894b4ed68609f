set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_small.py -x -q --timeout 200 --timeout-method thread -k "pinned_staging or concurrent" > gpurun_out/pin_tests.log 2>&1; rc=$?; echo "pin tests rc=$rc"; tail -2 gpurun_out/pin_tests.log; [ $rc -eq 0 ] || exit 1
DBSCAN_LIB_PATH=dbscan-on-spark_amd/lib_ab/tsm/libdbscan_hip.so timeout -k 10 500 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_batch.py -x -q --timeout 300 --timeout-method thread > gpurun_out/tsm_tests.log 2>&1; rc=$?; echo "tsm tests rc=$rc"; tail -2 gpurun_out/tsm_tests.log; [ $rc -eq 0 ] || exit 1
VARIANTS="main tsm" ROUNDS=2 BENCH_ARGS="--config 5 --steps 3 --warmup 1 --no-seam" bash tools/ab_bench.sh && VARIANTS="main tsm" ROUNDS=2 bash tools/ab_bench.sh
