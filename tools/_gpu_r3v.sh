set -o pipefail
mkdir -p gpurun_out/v
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/v/gputest.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/v/gputest.log; [ $rc -eq 0 ] || exit $rc
TAG=round3_m bash tools/round_evidence.sh
