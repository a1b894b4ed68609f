set -o pipefail
mkdir -p gpurun_out/c5
DBSCAN_TEST_FULL_SCALE=1 timeout -k 10 1170 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -v -s --timeout 1160 --timeout-method thread -k test_config5_full_size_train_node > gpurun_out/c5/test.log 2>&1
rc=$?; echo "c5 rc=$rc"; tail -15 gpurun_out/c5/test.log; free -g | head -3; exit $rc
