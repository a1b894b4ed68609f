set -o pipefail
mkdir -p gpurun_out/k
bash tools/profile.sh || exit 1
DBSCAN_NODE_TRACE=1 DBSCAN_TEST_FULL_SCALE=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -k config5_full_size_vs_oracle -s -v --timeout 580 --timeout-method thread > gpurun_out/k/c5.log 2>&1
rc=$?; echo "c5 rc=$rc"; tail -5 gpurun_out/k/c5.log; [ $rc -eq 0 ] || exit $rc
cp gpurun_out/config5_oracle_digest.json tests/golden/
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/k/test.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/k/test.log; exit $rc
