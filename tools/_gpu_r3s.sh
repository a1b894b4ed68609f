set -o pipefail
mkdir -p gpurun_out/s
timeout -k 10 300 python -u -m pytest tests/test_gpu_small.py tests/test_gpu_batch.py tests/test_gpu_parity.py tests/test_gpu_train.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/s/test.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/s/test.log; [ $rc -eq 0 ] || exit $rc
for v in stamps_old stamps_new; do
DBSCAN_LIB_PATH=dbscan-on-spark_amd/lib_ab/$v/libdbscan_hip.so timeout -k 10 120 python tools/small_stamps.py > gpurun_out/s/$v.txt 2>&1; echo "$v rc=$?"; grep "^m=" gpurun_out/s/$v.txt
done
