set -o pipefail
mkdir -p gpurun_out/o/profiles
DBSCAN_NODE_TRACE=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py -k "config5_full_size_train_node" -s -v --timeout 380 --timeout-method thread > gpurun_out/o/c5.log 2>&1
rc=$?; echo "c5 rc=$rc"; tail -4 gpurun_out/o/c5.log; [ $rc -eq 0 ] || exit $rc
bash tools/profile.sh || exit 1
PROF_DEST=gpurun_out/o/profiles python3 tools/pmc_summary.py gpurun_out/prof round3_l > gpurun_out/o/sum_c2.txt 2>&1 || exit 1
cp gpurun_out/prof/trace.log gpurun_out/o/trace_c2.log; rm -rf gpurun_out/prof
NO_PROFILE=1 bash tools/round_evidence.sh
