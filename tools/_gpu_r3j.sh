set -o pipefail
mkdir -p gpurun_out/j
timeout -k 10 300 python -u -m pytest tests/test_gpu_small.py tests/test_gpu_batch.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/j/test.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/j/test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 100 python tools/small_stamps.py > gpurun_out/j/stamps_note.log 2>&1; true
bash tools/profile.sh
