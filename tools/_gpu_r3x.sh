set -o pipefail
mkdir -p gpurun_out/x
timeout -k 10 300 python -u -m pytest tests/test_gpu_small.py tests/test_gpu_batch.py tests/test_gpu_parity.py tests/test_gpu_train.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/x/test.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/x/test.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do for v in st0 st1 st2; do
DBSCAN_LIB_PATH=dbscan-on-spark_amd/lib_ab/$v/libdbscan_hip.so timeout -k 10 120 python tools/small_stamps.py > gpurun_out/x/$v.$r.txt 2>&1 || exit 1; echo "$v"; grep "^m=" gpurun_out/x/$v.$r.txt
done; done
