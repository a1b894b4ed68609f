set -o pipefail
mkdir -p gpurun_out/g
timeout -k 10 300 python -u -m pytest tests/test_gpu_small.py tests/test_gpu_batch.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/g/test.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/g/test.log; [ $rc -eq 0 ] || exit $rc
DBSCAN_LIB_PATH=dbscan-on-spark_amd/lib_ab/stamps/libdbscan_hip.so timeout -k 10 200 python tools/small_stamps.py
