set -o pipefail
mkdir -p gpurun_out/e
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/e/gputest.log 2>&1
rc=$?; echo "gputest rc=$rc"; tail -4 gpurun_out/e/gputest.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/e/sprobe -o run -- python3 tools/small_probe.py > gpurun_out/e/sprobe.log 2>&1
rc=$?; echo "sprobe rc=$rc"; [ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/e/sprobe -name "*kernel_stats.csv" | head -1); head -12 "$f" | cut -c1-200
