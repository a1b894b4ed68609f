set -o pipefail
mkdir -p gpurun_out/r
timeout -k 10 300 python -u -m pytest tests/test_gpu_bucket.py tests/test_gpu_parity.py tests/test_gpu_structure.py tests/test_gpu_batch.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r/test.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r/test.log; [ $rc -eq 0 ] || exit $rc
VARIANTS="old main" ROUNDS=2 BENCH_ARGS="--config 5 --steps 3 --warmup 1 --no-seam" bash tools/ab_bench.sh || exit 1
VARIANTS="old main" ROUNDS=2 BENCH_ARGS="--steps 20 --warmup 5 --no-seam" bash tools/ab_bench.sh || exit 1
grep -h -o '"bin": [0-9.]*\|"msd_upsweep": [0-9.]*\|"radix_upsweep<8>": [0-9.]*' gpurun_out/ab/*.log
DBSCAN_LIB_PATH=dbscan-on-spark_amd/lib_ab/stamps/libdbscan_hip.so timeout -k 10 120 python tools/small_stamps.py > gpurun_out/r/stamps.txt 2>&1; echo "stamps rc=$?"; tail -12 gpurun_out/r/stamps.txt
