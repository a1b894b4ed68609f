set -o pipefail
mkdir -p gpurun_out/z
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/z/gputest.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/z/gputest.log; [ $rc -eq 0 ] || exit $rc
TAG=round3_n bash tools/round_evidence.sh
